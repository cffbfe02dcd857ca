#!/bin/bash
# The level kernel (a lane group per env, one lane per node of a level: DESIGN §6.6) on ntom,
# timed and with its HBM traffic (FETCH_SIZE / WRITE_SIZE passes), beside the staged kernel.
#   tools/gpu_level_ntom.sh TAG
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out/level_$1; mkdir -p "$OUT"
for k in staged level; do
  timeout -k 10 300 python tools/bench_sc.py --no-cpu-baseline --scenario ntom --kernel $k --steps 20 > "$OUT/bench_$k.log" 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$OUT/$C" -o pmc -- \
      python3 "$ROOT/tools/bench_sc.py" --no-cpu-baseline --steps 4 --warmup 1 --scenario ntom --kernel level \
      > "$OUT/$C.log" 2>&1 || exit 1
done
echo ok
