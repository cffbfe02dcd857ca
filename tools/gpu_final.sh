#!/bin/bash
# The final-tree evidence in one call: BeerGame PMC passes and their keyed summary (written to
# profiles/ first, so the bench lines of this same call find their traffic), the SupplyChain
# evidence (tools/gpu_sc_evidence.sh), then the GPU tests, smoke, bench (defaults, the driver's
# configuration, the one-rank RCCL rehearsal), rocprofv3 stats and the drop-in env latencies.
#   tools/gpu_final.sh TAG   (via gpurun)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=${1:-r05zz}
bash tools/gpu_session.sh ${TAG} pmc || exit 1
python tools/pmc_summary.py gpurun_out/pmc_${TAG} --meta bench=beergame-v0 n_envs=65536 --family bg > profiles/${TAG}_pmc_summary.json || exit 1
cp profiles/${TAG}_pmc_summary.json gpurun_out/
bash tools/gpu_sc_evidence.sh ${TAG} || exit 1
bash tools/gpu_session.sh ${TAG} tests,smoke,bench,pg,prof || exit 1
timeout -k 10 300 python tools/facade_latency.py > gpurun_out/facade_latency_${TAG}.log 2>&1 || exit 1
timeout -k 10 200 python tools/server_latency_probe.py > gpurun_out/server_probe_${TAG}.log 2>&1 || exit 1
echo final ok
