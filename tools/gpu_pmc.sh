#!/bin/bash
# PMC passes (counters only: no sys/runtime tracing with --pmc). FETCH_SIZE and
# WRITE_SIZE need separate passes on gfx950 (TCC slots). Each pass runs a short bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_${1:-r01}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
pass() {  # name, counters, command...
  local name=$1 ctr=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/$name" -o pmc -- "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "pass $name ($ctr) rc=$rc"; return $rc
}
BG="python3 $ROOT/bench.py --no-cpu-baseline --steps 700 --warmup 70"
SC="python3 $ROOT/tools/bench_sc.py --no-cpu-baseline --steps 10 --warmup 2"
pass bg_fetch FETCH_SIZE $BG && \
pass bg_write WRITE_SIZE $BG && \
pass bg_sq "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" $BG && \
pass sc_fetch FETCH_SIZE $SC && \
pass sc_write WRITE_SIZE $SC && \
pass sc_sq "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" $SC && \
pass sc_cache "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_SALU SQ_INSTS_SMEM" $SC
