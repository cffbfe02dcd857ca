#!/bin/bash
# A/B timing of experiment builds (tools/exp_build.py): bench.py per BeerGame variant,
# bench_sc.py per SupplyChain variant. Usage: tools/gpu_exp.sh TAG "bgvariants" "scvariants" [sc-args]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out; TAG=$1; mkdir -p $OUT
LOG=$OUT/exp_$TAG.log; : > $LOG
for v in $2; do
  root=gym-supplychain_amd; [ "$v" != base ] && root=exp/$v
  SCG_PKG_ROOT=$root timeout -k 10 120 python bench.py --no-cpu-baseline $BENCH_ARGS > $OUT/exp_${TAG}_$v.log 2>&1
  rc=$?; echo "bg $v rc=$rc $(grep -o '"value": [0-9.e+]*\|"avg_kernel_us": [0-9.]*' $OUT/exp_${TAG}_$v.log | tr '\n' ' ')" | tee -a $LOG
  [ $rc -ne 0 ] && exit $rc
done
for v in $3; do
  root=gym-supplychain_amd; [ "$v" != base ] && root=exp/$v
  SCG_PKG_ROOT=$root timeout -k 10 300 python tools/bench_sc.py --no-cpu-baseline $4 > $OUT/exp_${TAG}_sc_$v.log 2>&1
  rc=$?; echo "sc $v rc=$rc $(grep -o '"kernel": "[a-z]*"\|"avg_kernel_us": [0-9.]*' $OUT/exp_${TAG}_sc_$v.log | tr '\n' ' ')" | tee -a $LOG
  [ $rc -ne 0 ] && exit $rc
done
exit 0
