#!/bin/bash
# Final-tree evidence after a SupplyChain-only source change (the BeerGame sources, and so
# their keyed PMC summary and bench lines, unchanged): the SupplyChain evidence
# (tools/gpu_sc_evidence.sh), the whole GPU suite, smoke and the drop-in env latencies.
#   tools/gpu_final_sc.sh TAG   (via gpurun)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=${1:-r06zb}
bash tools/gpu_sc_evidence.sh ${TAG} || exit 1
bash tools/gpu_session.sh ${TAG} tests,smoke || exit 1
timeout -k 10 300 python tools/facade_latency.py > gpurun_out/facade_latency_${TAG}.log 2>&1 || exit 1
timeout -k 10 200 python tools/server_latency_probe.py > gpurun_out/server_probe_${TAG}.log 2>&1 || exit 1
echo final-sc ok
