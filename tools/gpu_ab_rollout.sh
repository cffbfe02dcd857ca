#!/bin/bash
# BeerGame rollout/step A/B over tools/sweep_bg.py (base = in-tree, NAME = exp/NAME).
#   tools/gpu_ab_rollout.sh TAG "base v1 ..." [MIN_LOG2] [MAX_LOG2]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out; TAG=$1; mkdir -p $OUT; LOG=$OUT/abro_$TAG.log; : > $LOG
for v in $2; do
  root=gym-supplychain_amd; [ "$v" != base ] && root=exp/$v
  echo "== $v" >> $LOG
  SCG_PKG_ROOT=$root timeout -k 10 200 python tools/sweep_bg.py --min-log2 ${3:-16} --max-log2 ${4:-18} \
      2>&1 | grep '^{' >> $LOG || exit 1
done
cat $LOG
