#!/bin/bash
# SupplyChain GPU session: parity tests for SC, bench_sc, rocprofv3 kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${1:-sc}
mkdir -p "$OUT"
timeout -k 10 600 python -m pytest tests/test_gpu_supplychain.py -x -q > "$OUT/pytest_sc_$TAG.log" 2>&1
rc=$?; echo "pytest sc rc=$rc"; tail -3 "$OUT/pytest_sc_$TAG.log"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python tools/bench_sc.py > "$OUT/bench_sc_$TAG.log" 2>&1
rc=$?; echo "bench_sc rc=$rc"; cat "$OUT/bench_sc_$TAG.log" | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_sc_$TAG" -o bench_sc -- \
    python3 "$ROOT/tools/bench_sc.py" --no-cpu-baseline --steps 20 > "$OUT/prof_sc_$TAG.log" 2>&1
rc=$?; echo "rocprofv3 rc=$rc"; exit $rc
