#!/bin/bash
# Instruction-fetch counters of the SupplyChain auto kernels (one rocprofv3 --pmc pass each).
#   tools/gpu_icache.sh TAG [SCENARIO]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out/icache_$1; mkdir -p "$OUT"; SCN=${2:-both}
cd /tmp && export TMPDIR=/tmp
n=0
for C in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_VALU"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/p$n" -o pmc -- \
      python3 "$ROOT/tools/bench_sc.py" --no-cpu-baseline --steps 4 --warmup 1 --scenario $SCN --kernel auto \
      > "$OUT/p$n.log" 2>&1 || exit 1
  echo "pass $n ok"
done
