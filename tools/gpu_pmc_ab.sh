#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes of one SupplyChain scenario for the tree and exp/ variants
# (one pass per counter and variant; summaries with tools/pmc_summary.py afterwards).
#   tools/gpu_pmc_ab.sh TAG SCENARIO KERNEL "base v1 ..."
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd); TAG=$1; SCN=$2; KERN=$3; VARS=$4
cd /tmp && export TMPDIR=/tmp
for v in $VARS; do
  PM=$ROOT/gpurun_out/pmcab_${TAG}/$v; mkdir -p "$PM"
  if [ "$v" = base ]; then unset SCG_PKG_ROOT; else export SCG_PKG_ROOT=$ROOT/exp/$v; fi
  SC="python3 $ROOT/tools/bench_sc.py --no-cpu-baseline --steps 6 --warmup 1 --scenario $SCN --kernel $KERN"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$PM/sc_fetch" -o pmc -- $SC > "$PM/sc_fetch.log" 2>&1 || { echo "fetch $v failed"; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$PM/sc_write" -o pmc -- $SC > "$PM/sc_write.log" 2>&1 || { echo "write $v failed"; exit 1; }
  echo "pmc $v ok"
done
