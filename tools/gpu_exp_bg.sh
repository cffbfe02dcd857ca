#!/bin/bash
# BeerGame A/B: per variant, bench.py (back-to-back launches) and floor_probe.py at 1,024
# and 65,536 envs (isolated launches). Usage: tools/gpu_exp_bg.sh TAG "v1 v2 ..." (base = in-tree)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out; TAG=$1; mkdir -p $OUT; LOG=$OUT/expbg_$TAG.log; : > $LOG
for v in $2; do
  root=gym-supplychain_amd; [ "$v" != base ] && root=exp/$v
  SCG_PKG_ROOT=$root timeout -k 10 120 python bench.py --no-cpu-baseline --steps 7000 > $OUT/expbg_${TAG}_$v.log 2>&1 || exit 1
  SCG_PKG_ROOT=$root timeout -k 10 120 python tools/floor_probe.py --min-log2 10 --max-log2 10 > $OUT/expbg_${TAG}_${v}_f.log 2>&1 || exit 1
  SCG_PKG_ROOT=$root timeout -k 10 120 python tools/floor_probe.py --min-log2 16 --max-log2 16 >> $OUT/expbg_${TAG}_${v}_f.log 2>&1 || exit 1
  python - "$v" $OUT/expbg_${TAG}_$v.log $OUT/expbg_${TAG}_${v}_f.log >> $LOG <<'PY'
import json, sys
b = [json.loads(l) for l in open(sys.argv[2]) if l.startswith("{")][0]
f = [json.loads(l) for l in open(sys.argv[3]) if l.startswith("{")]
print(sys.argv[1], "value %.3e" % b["value"], "b2b_kernel_us %.2f" % b["roofline"]["avg_kernel_us"],
      " ".join("N=%d iso %.2f b2b %.2f wall %.2f" % (x["n_envs"], x["step_isolated_us"], x["step_back_to_back_us"],
                                                      x["step_wall_us"]) for x in f))
PY
  tail -n 1 $LOG
done
exit 0
