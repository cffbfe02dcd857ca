#!/bin/bash
# The step-server GPU tests and latency logs (via gpurun): tests/test_gpu_step_server.py and
# the drop-in facade tests, then tools/facade_latency.py (1 env and 8 envs round-robin) and
# tools/server_latency_probe.py. Every GPU step has its own time limit; a failure stops.
#   tools/gpu_server_check.sh TAG
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=${1:-r06}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_step_server.py tests/test_gpu_beergame.py -m gpu -x -v \
    --timeout 120 --timeout-method thread > $OUT/server_tests_$TAG.log 2>&1 || { tail -40 $OUT/server_tests_$TAG.log; exit 1; }
tail -3 $OUT/server_tests_$TAG.log
timeout -k 10 300 python tools/facade_latency.py --bg-episodes 100 --sc-episodes 2 > $OUT/facade_latency_$TAG.log 2>&1 || { tail -20 $OUT/facade_latency_$TAG.log; exit 1; }
cut -c1-260 $OUT/facade_latency_$TAG.log
timeout -k 10 200 python tools/server_latency_probe.py > $OUT/server_probe_$TAG.log 2>&1 || { tail -20 $OUT/server_probe_$TAG.log; exit 1; }
cut -c1-260 $OUT/server_probe_$TAG.log
echo server ok
