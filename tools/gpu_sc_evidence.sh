#!/bin/bash
# Final-tree SupplyChain evidence in one call: PMC passes per scenario, their summaries
# (written to profiles/ for bench_sc's keyed lookup and copied to gpurun_out/), then bench_sc
# with same-host CPU baselines and the ledger runs.   tools/gpu_sc_evidence.sh TAG (via gpurun)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=${1:-r04zd}
bash tools/gpu_session.sh ${TAG} scpmc || exit 1
for scn in 2perstage 2perstage_mp ntom; do
  N=65536; [ $scn = ntom ] && N=262144
  python tools/pmc_summary.py gpurun_out/scpmc_${TAG}/$scn --meta bench=bench_sc scenario=$scn n_envs=$N kernel=auto build_info=false --family sc > profiles/${TAG}_sc_${scn}_pmc_summary.json || exit 1
  cp profiles/${TAG}_sc_${scn}_pmc_summary.json gpurun_out/
done
bash tools/gpu_session.sh ${TAG} sc || exit 1
timeout -k 10 400 python tools/bench_sc.py --scenario both --kernel auto --build-info --no-cpu-baseline > gpurun_out/bench_sc_ledgers_${TAG}.log 2>&1 || exit 1
echo ok
