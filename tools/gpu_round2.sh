#!/bin/bash
# Round-2 GPU session: parity tests, smoke, bench (full line), rocprofv3 kernel stats of the
# bench, PMC traffic passes of the step kernel, SupplyChain bench. Every GPU step has its own
# time limit and a failure stops the script.
#   tools/gpu_round2.sh TAG [skip-tests]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${1:-r02}
mkdir -p "$OUT"
stop() { echo "step '$1' ended with $2: stopping"; exit "$2"; }
run() {  # run NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -v amdgpu.ids "$OUT/${name}_$TAG.log" | tail -3 | cut -c1-600
  [ $rc -ne 0 ] && stop "$name" $rc
  return 0
}
if [ "$2" != "skip-tests" ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
run bench 400 python bench.py
run bench_driver 300 python bench.py --steps 20 --warmup 5
run bench_sc 600 python tools/bench_sc.py --kernel both --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o bench -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --no-extras > "$OUT/prof_$TAG.log" 2>&1
rc=$?; echo "rocprofv3 rc=$rc"; [ $rc -ne 0 ] && stop rocprof $rc
PM=$OUT/pmc_$TAG; mkdir -p $PM
BG="python3 $ROOT/bench.py --no-cpu-baseline --no-extras --steps 700 --warmup 70"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$PM/bg_fetch" -o pmc -- $BG > "$PM/bg_fetch.log" 2>&1 || stop pmc_fetch $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$PM/bg_write" -o pmc -- $BG > "$PM/bg_write.log" 2>&1 || stop pmc_write $?
echo "pmc ok"
exit 0
