#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter per rocprofv3 run) of the SupplyChain bench,
# for the in-tree build ("base") and experiment builds (exp/NAME from tools/exp_build.py),
# then one timing run per variant.
#   tools/gpu_sc_traffic.sh TAG [SCENARIO] [KERNEL] [VARIANTS...]    (default: both auto base)
# Summaries: python tools/pmc_summary.py gpurun_out/sctraffic_TAG/VARIANT
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd); TAG=$1; SCN=${2:-both}; KERN=${3:-auto}; shift 3 2>/dev/null; VARS=${*:-base}
cd /tmp && export TMPDIR=/tmp
for v in $VARS; do
  PM=$ROOT/gpurun_out/sctraffic_$TAG/$v; mkdir -p "$PM"
  pkg=$ROOT/gym-supplychain_amd; [ "$v" != base ] && pkg=$ROOT/exp/$v
  for c in FETCH_SIZE WRITE_SIZE; do
    d=sc_fetch; [ $c = WRITE_SIZE ] && d=sc_write
    SCG_PKG_ROOT=$pkg timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$PM/$d" -o pmc -- \
      python3 "$ROOT/tools/bench_sc.py" --no-cpu-baseline --steps 6 --warmup 1 --scenario $SCN --kernel $KERN \
      > "$PM/$d.log" 2>&1 || { echo "$v $c failed"; exit 1; }
  done
  SCG_PKG_ROOT=$pkg timeout -k 10 300 python3 "$ROOT/tools/bench_sc.py" --no-cpu-baseline --scenario $SCN --kernel $KERN \
    > "$PM/time.log" 2>&1 || { echo "$v timing failed"; exit 1; }
  echo "$v ok"
done
