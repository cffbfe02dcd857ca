#!/bin/bash
# SupplyChain A/B on the auto kernels: the SupplyChain GPU parity tests on the in-tree build,
# then tools/bench_sc.py --kernel auto for each variant in turn, REPS times (alternating).
#   tools/gpu_ab_auto.sh TAG "base v1 ..." [REPS] [TESTS]   (base = in-tree, v = exp/v)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=$1; VARS=${2:-base}; REPS=${3:-2}; TESTS=${4:-tests/test_gpu_supplychain.py}
if [ "$TESTS" != none ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1
  rc=$?; tail -2 gpurun_out/pt_$TAG.log; [ $rc -ne 0 ] && exit $rc
fi
for r in $(seq 1 "$REPS"); do
  for v in $VARS; do
    root=gym-supplychain_amd; [ "$v" != base ] && root=exp/$v
    SCG_PKG_ROOT=$root timeout -k 10 300 python tools/bench_sc.py --no-cpu-baseline --kernel auto > gpurun_out/sc_${TAG}_${v}_$r.log 2>&1 || exit 1
    grep '^{' gpurun_out/sc_${TAG}_${v}_$r.log | python -c "
import json,sys
for l in sys.stdin:
  d=json.loads(l); print('$v', d['config']['workload'][:22], d['config']['kernel'], 'kern_us %.1f'%d['roofline']['avg_kernel_us'], 'frac %.3f'%d['roofline']['frac'])"
  done
done
