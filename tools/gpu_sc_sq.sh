#!/bin/bash
# SQ/TA/TD counter passes over one SupplyChain kernel (latency analysis), one pass per run.
#   tools/gpu_sc_sq.sh TAG SCENARIO KERNEL [PKG_ROOT]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out/scpmc3_$1; mkdir -p "$OUT"
[ -n "$4" ] && export SCG_PKG_ROOT=$ROOT/$4
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_ACTIVE_INST_ANY TD_TD_BUSY TD_TC_STALL"
n=0
P4="SQ_WAVES SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_SCA"
for C in "$P1" "$P2" "$P3" "$P4"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/p$n" -o pmc -- \
      python3 "$ROOT/tools/bench_sc.py" --no-cpu-baseline --steps 4 --warmup 1 --scenario $2 --kernel $3 \
      > "$OUT/p$n.log" 2>&1 || exit 1
  echo "pass $n ok"
done
