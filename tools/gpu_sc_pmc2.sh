#!/bin/bash
# SQ counters of the SupplyChain kernels, one scenario and kernel per pass.
#   tools/gpu_sc_pmc2.sh TAG SCENARIO "kernels"
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out/scpmc2_$1; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
for k in $3; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/$k" -o pmc -- \
      python3 "$ROOT/tools/bench_sc.py" --no-cpu-baseline --steps 4 --warmup 1 --scenario $2 --kernel $k \
      > "$OUT/$k.log" 2>&1 || exit 1
  echo "pass $k ok"
done
