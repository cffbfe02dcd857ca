#!/bin/bash
# Instruction-cache and wait counters over one SupplyChain kernel, one pass per run.
#   tools/gpu_sc_icache.sh TAG SCENARIO KERNEL
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out/scic_$1; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
n=0
for C in "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/p$n" -o pmc -- \
      python3 "$ROOT/tools/bench_sc.py" --no-cpu-baseline --steps 4 --warmup 1 --scenario $2 --kernel $3 \
      > "$OUT/p$n.log" 2>&1 || { echo "pass $n failed"; tail -5 "$OUT/p$n.log"; exit 1; }
  echo "pass $n ok"
done
