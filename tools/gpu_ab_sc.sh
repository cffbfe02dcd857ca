#!/bin/bash
# SupplyChain A/B: GPU parity tests on the in-tree build, then tools/bench_sc.py per variant
# (base = in-tree, NAME = exp/NAME from tools/exp_build.py).  tools/gpu_ab_sc.sh TAG "base v1 ..." [KERNEL]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=$1; VARS=${2:-base}; KERN=${3:-all}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pt_$TAG.log; [ $rc -ne 0 ] && exit $rc
for v in $VARS; do
  root=gym-supplychain_amd; [ $v != base ] && root=exp/$v
  SCG_PKG_ROOT=$root timeout -k 10 300 python tools/bench_sc.py --no-cpu-baseline --kernel $KERN > gpurun_out/sc_${TAG}_$v.log 2>&1 || exit 1
  echo "== $v"; grep '^{' gpurun_out/sc_${TAG}_$v.log | python -c "
import json,sys
for l in sys.stdin:
  d=json.loads(l); print(d['config']['workload'][:22], d['config']['kernel'], '%.3e'%d['value'], 'kern_us %.1f'%d['roofline']['avg_kernel_us'], 'frac %.3f'%d['roofline']['frac'])"
done
