#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the BeerGame step kernel at 1,048,576 envs (past the Infinity Cache).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd); PM=$ROOT/gpurun_out/pmc1m_$1; mkdir -p $PM
cd /tmp && export TMPDIR=/tmp
BG="python3 $ROOT/bench.py --envs 1048576 --no-cpu-baseline --no-extras --steps 70 --warmup 35 --kernel-samples 35"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$PM/bg_fetch" -o pmc -- $BG > "$PM/bg_fetch.log" 2>&1 || { echo fetch failed; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$PM/bg_write" -o pmc -- $BG > "$PM/bg_write.log" 2>&1 || { echo write failed; exit 1; }
grep '^{' "$PM/bg_fetch.log" | cut -c1-200
echo pmc ok
