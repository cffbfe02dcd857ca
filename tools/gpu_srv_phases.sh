#!/bin/bash
# SupplyChain step-server phase clocks (tools/sc_server_phase_probe.py) for stamp builds,
# alternated: gpu_srv_phases.sh OUT_LOG VARIANT...
set -o pipefail
out=$1; shift
echo "# SupplyChain step server phases: $* (tools/sc_server_phase_probe.py, two alternations)" > "$out"
for rep in 1 2; do
  for v in "$@"; do
    echo "== $v $rep" >> "$out"
    SCG_PKG_ROOT=exp/$v timeout -k 10 180 python -u tools/sc_server_phase_probe.py >> "$out" 2>&1 || exit $?
  done
done
