#!/bin/bash
# Timing-only A/B of library variants on one SupplyChain scenario (no parity tests: for
# experiment builds from tools/exp_build.py).  tools/gpu_ab_quick.sh TAG "base v1 ..." SCENARIO KERNEL [ROUNDS] [EXTRA]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=$1; VARS=${2:-base}; SCN=${3:-2perstage}; KERN=${4:-nodes}; ROUNDS=${5:-2}; EXTRA=$6
for r in $(seq 1 $ROUNDS); do
  for v in $VARS; do
    root=gym-supplychain_amd; [ $v != base ] && root=exp/$v
    SCG_PKG_ROOT=$root timeout -k 10 200 python tools/bench_sc.py --no-cpu-baseline --scenario $SCN --kernel $KERN \
        --steps 100 $EXTRA > gpurun_out/q_${TAG}_${v}_$r.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/q_${TAG}_${v}_$r.log; exit 1; }
    echo -n "== $r $v "; grep '^{' gpurun_out/q_${TAG}_${v}_$r.log | python -c "
import json,sys
for l in sys.stdin:
  d=json.loads(l); print(d['config']['kernel'], 'kern_us %.2f'%d['roofline']['avg_kernel_us'], 'frac %.3f'%d['roofline']['frac'])"
  done
done
