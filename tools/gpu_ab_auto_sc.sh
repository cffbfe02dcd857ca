#!/bin/bash
# SupplyChain A/B of the auto kernels: tools/bench_sc.py per variant (base = in-tree, NAME =
# exp/NAME from tools/exp_build.py), REPS alternations, timing only (no parity check: an
# ablation variant may change the dynamics).  tools/gpu_ab_auto_sc.sh TAG "base v1 ..." [REPS] [SCENARIO]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=$1; VARS=${2:-base}; REPS=${3:-2}; SCN=${4:-all}
for r in $(seq 1 "$REPS"); do
  for v in $VARS; do
    root=gym-supplychain_amd; [ "$v" != base ] && root=exp/$v
    SCG_BENCH_NO_CHECK=1 SCG_PKG_ROOT=$root timeout -k 10 300 python tools/bench_sc.py --no-cpu-baseline --kernel auto \
      --scenario "$SCN" > "gpurun_out/abs_${TAG}_${v}_$r.log" 2>&1 || { echo "$v failed"; tail -n 5 "gpurun_out/abs_${TAG}_${v}_$r.log"; exit 1; }
    echo "== $v rep $r"; grep '^{' "gpurun_out/abs_${TAG}_${v}_$r.log" | python -c "
import json,sys
for l in sys.stdin:
  d=json.loads(l); print(d['config']['workload'][:28], d['config']['kernel'], 'kern_us %.1f'%d['roofline']['avg_kernel_us'], 'frac %.3f'%d['roofline']['frac'])"
  done
done
