#!/bin/bash
# SupplyChain GPU parity, then tree vs exp/prev on both configs, then FETCH/WRITE PMC of the tree.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out/dirty_$1; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_supplychain.py -x -q --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for v in tree prev; do
  if [ "$v" = tree ]; then pk=""; else pk="$ROOT/exp/$v"; fi
  SCG_PKG_ROOT=$pk timeout -k 10 300 python tools/bench_sc.py --no-cpu-baseline --steps 40 > $OUT/bench_$v.log 2>&1 || { tail -5 $OUT/bench_$v.log; exit 1; }
  grep '^{' $OUT/bench_$v.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']; print('$v', d['config']['workload'][:22], d['config']['kernel'], round(r['avg_kernel_us'],1), 'us', round(r['frac'],3))"
done
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o pmc -- \
    python3 "$ROOT/tools/bench_sc.py" --no-cpu-baseline --steps 6 --warmup 1 > "$OUT/pmc_$c.log" 2>&1 || { echo "pmc $c failed"; exit 1; }
done
echo pmc ok
