#!/bin/bash
# Quick GPU session: full GPU tests, then the bench at the driver's and the default config.
#   tools/gpu_quick.sh TAG
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out
TAG=${1:-quick}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu_$TAG.log"
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> "$OUT/bench_driver_$TAG.log" 2>&1 || exit $?
done
tail -3 "$OUT/bench_driver_$TAG.log"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_$TAG.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 "$OUT/bench_$TAG.log"
exit $rc
