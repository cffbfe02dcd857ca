#!/bin/bash
# BeerGame bench A/B of the tree against one exp/ library variant (3 rounds, one box).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in base prevsrv; do
    root=gym-supplychain_amd; [ $v != base ] && root=exp/$v
    SCG_PKG_ROOT=$root timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras > gpurun_out/bgab_${v}_$r.log 2>&1 || { echo FAIL $v; tail -5 gpurun_out/bgab_${v}_$r.log; exit 1; }
    echo -n "== $r $v "; grep '^{' gpurun_out/bgab_${v}_$r.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print('value %.3e kern_us %.3f'%(d['value'], d['roofline']['avg_kernel_us']))"
  done
done
