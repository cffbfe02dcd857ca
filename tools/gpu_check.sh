#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel stats. Each GPU step has
# its own time limit; a crash/fault/timeout (exit > 1) stops the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${1:-r01}
mkdir -p "$OUT"
stop() { echo "step '$1' ended with $2: stopping"; exit "$2"; }

timeout -k 10 600 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest -m gpu rc=$rc"; tail -3 "$OUT/pytest_gpu_$TAG.log"
[ $rc -gt 1 ] && stop pytest $rc

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke_$TAG.log"
[ $rc -ne 0 ] && stop smoke $rc

timeout -k 10 400 python bench.py > "$OUT/bench_$TAG.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 "$OUT/bench_$TAG.log"
[ $rc -ne 0 ] && stop bench $rc

cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o bench -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline > "$OUT/prof_$TAG.log" 2>&1
rc=$?; echo "rocprofv3 rc=$rc"; tail -2 "$OUT/prof_$TAG.log"
[ $rc -ne 0 ] && stop rocprof $rc
find "$OUT/prof_$TAG" -name '*stats*' | head
exit 0
