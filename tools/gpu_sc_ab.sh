#!/bin/bash
# SupplyChain kernel A/B on the GPU box: tools/bench_sc.py for the tree and each exp/
# variant, then SQ counter passes of the tree's step kernels (one rocprofv3 --pmc run each).
#   tools/gpu_sc_ab.sh TAG [VARIANT ...]      (VARIANT = a directory name under exp/)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/sc_$1
shift
mkdir -p "$OUT"
stop() { echo "step '$1' ended with $2: stopping"; exit "$2"; }
for v in tree "$@"; do
  if [ "$v" = tree ]; then pk=""; else pk="$ROOT/exp/$v"; fi
  SCG_PKG_ROOT=$pk timeout -k 10 300 python tools/bench_sc.py --no-cpu-baseline --steps 60 > "$OUT/bench_$v.log" 2>&1
  rc=$?; echo "bench $v rc=$rc"; grep '^{' "$OUT/bench_$v.log" | cut -c1-400
  [ $rc -ne 0 ] && { tail -5 "$OUT/bench_$v.log"; stop "bench $v" $rc; }
done
[ -n "$SC_NO_PMC" ] && exit 0
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS"
P2="SQ_INSTS_SMEM,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS"
for sc in 2perstage ntom; do
  i=0
  for pm in $P1 $P2; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $pm --output-format csv -d "$OUT/pmc_${sc}_$i" -o pmc -- \
      python3 "$ROOT/tools/bench_sc.py" --no-cpu-baseline --scenario $sc --steps 20 --warmup 3 > "$OUT/pmc_${sc}_$i.log" 2>&1 \
      || stop "pmc $sc $i" $?
  done
done
echo "pmc ok"
