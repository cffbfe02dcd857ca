#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the auto-chosen SupplyChain kernels at the BASELINE sizes.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd); PM=$ROOT/gpurun_out/sctraffic_$1; mkdir -p $PM
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$PM/$c" -o pmc -- \
    python3 "$ROOT/tools/bench_sc.py" --no-cpu-baseline --steps 6 --warmup 1 > "$PM/$c.log" 2>&1 || { echo "$c failed"; exit 1; }
done
echo pmc ok
