#!/bin/bash
# SQ counters of the node-parallel kernel on sc-2perstage-v0 (one rocprofv3 --pmc run each).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out/npmc_$1; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS"
P2="SQ_INSTS_SMEM,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS,SQ_BUSY_CYCLES"
i=0
for pm in $P1 $P2; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pm --output-format csv -d "$OUT/p$i" -o pmc -- \
    python3 "$ROOT/tools/bench_sc.py" --no-cpu-baseline --scenario 2perstage --kernel nodes --steps 20 --warmup 3 > "$OUT/p$i.log" 2>&1 \
    || { echo "pmc $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
echo pmc ok
