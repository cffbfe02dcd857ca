#!/bin/bash
# One full GPU session: parity tests, smoke, bench, SupplyChain bench (both kernels),
# BeerGame kernel variants, rocprofv3 kernel stats of bench.py. Every GPU step runs under
# its own time limit; a crash/fault/timeout stops the script (no further GPU step).
#   tools/gpu_round.sh TAG [skip-tests]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${1:-r01}
mkdir -p "$OUT"
stop() { echo "step '$1' ended with $2: stopping"; exit "$2"; }
run() {  # run NAME SECONDS CMD... ; output to $OUT/NAME_$TAG.log
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -v amdgpu.ids "$OUT/${name}_$TAG.log" | tail -4
  [ $rc -ne 0 ] && stop "$name" $rc
  return 0
}

if [ "$2" != "skip-tests" ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
fi
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python bench.py
run bench_sc 600 python tools/bench_sc.py --kernel both --no-cpu-baseline
run bg_variants 300 python tools/bg_variants.py

cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o bench -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline > "$OUT/prof_$TAG.log" 2>&1
rc=$?; echo "rocprofv3 rc=$rc"; tail -2 "$OUT/prof_$TAG.log"
[ $rc -ne 0 ] && stop rocprof $rc
find "$OUT/prof_$TAG" -name '*stats*'
exit 0
