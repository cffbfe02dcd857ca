#!/bin/bash
# SQ counter passes over the SupplyChain step kernels (both kernels, configs 3 and 4).
# Counters only (no sys/runtime tracing with --pmc); each pass is its own short run.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out/scpmc_${1:-r01}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1
pass() {  # name, counters, args...
  local name=$1 ctr=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/$name" -o pmc -- \
      python3 "$ROOT/tools/bench_sc.py" --no-cpu-baseline --steps 6 --warmup 1 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "pass $name rc=$rc"; return $rc
}
A="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD"
B="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"
pass a_both "$A" --kernel both && pass b_both "$B" --kernel both && \
pass fetch FETCH_SIZE --kernel both && pass write WRITE_SIZE --kernel both
