#!/bin/bash
# SupplyChain: bench every kernel on both configs, then SQ counter passes of the level
# kernel on sc-2perstage-v0 (one rocprofv3 --pmc run each).  tools/gpu_sc_kernels.sh TAG
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/sck_$1
mkdir -p "$OUT"
stop() { echo "step '$1' ended with $2: stopping"; exit "$2"; }
timeout -k 10 400 python tools/bench_sc.py --no-cpu-baseline --steps 60 --kernel all > "$OUT/bench_all.log" 2>&1 \
  || { tail -5 "$OUT/bench_all.log"; stop bench $?; }
grep '^{' "$OUT/bench_all.log" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config'].get('workload','')[:40], d['config'].get('kernel'), round(d['roofline']['avg_kernel_us'],1), 'us kernel', round(d['ms_per_step']*1e3,1), 'us wall', d.get('roofline',{}).get('frac'))"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS"
P2="SQ_INSTS_SMEM,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS"
i=0
for pm in $P1 $P2; do
  i=$((i+1))
  for k in auto level; do
    timeout -s KILL 120 rocprofv3 --pmc $pm --output-format csv -d "$OUT/pmc_${k}_$i" -o pmc -- \
      python3 "$ROOT/tools/bench_sc.py" --no-cpu-baseline --scenario 2perstage --kernel $k --steps 20 --warmup 3 > "$OUT/pmc_${k}_$i.log" 2>&1 \
      || stop "pmc $k $i" $?
  done
done
echo "pmc ok"
