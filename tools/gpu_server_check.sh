#!/bin/bash
# Step-server check on the box: the BeerGame facade tests, the server latency probe, then the
# facade latency tool (server, launch path, round-4 design, the SupplyChain facade).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=${1:-r05x}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_beergame.py -x -v --timeout 120 --timeout-method thread -k "facade or overflow or single or server" > gpurun_out/srv_${TAG}_tests.log 2>&1; rc=$?; tail -15 gpurun_out/srv_${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/server_latency_probe.py > gpurun_out/srv_${TAG}_probe.log 2>&1; rc=$?; cat gpurun_out/srv_${TAG}_probe.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/facade_latency.py --bg-episodes 100 --sc-episodes 1 --no-cpu > gpurun_out/srv_${TAG}_latency.log 2>&1; rc=$?; cut -c1-300 gpurun_out/srv_${TAG}_latency.log; exit $rc
