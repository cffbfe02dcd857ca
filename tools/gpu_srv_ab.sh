#!/bin/bash
# Step-server latency A/B (tools/server_latency_probe.py) over exp/ variants, alternated;
# then the SupplyChain server's per-phase clocks from the stamp build (exp/nstamps).
#   gpu_srv_ab.sh OUT_LOG VARIANT... (each an exp/ directory name)
set -o pipefail
out=$1; shift
echo "# step-server latency A/B: $* (tools/server_latency_probe.py --weeks 1750 --sc-steps 720, two alternations)" > "$out"
for rep in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    echo "== $v $rep" >> "$out"
    SCG_PKG_ROOT=exp/$v timeout -k 10 240 python -u tools/server_latency_probe.py --weeks 1750 --sc-steps 720 >> "$out" 2>&1 || exit $?
  done
done
if [ -d exp/nstamps ]; then
  echo "== nstamps phases" >> "$out"
  SCG_PKG_ROOT=exp/nstamps timeout -k 10 240 python -u tools/sc_server_phase_probe.py >> "$out" 2>&1 || exit $?
fi
