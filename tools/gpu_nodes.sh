#!/bin/bash
# Node-parallel SupplyChain kernel: its GPU parity tests, then sc-2perstage bench of every
# kernel.  tools/gpu_nodes.sh TAG
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/nodes_$1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_supplychain.py -x -v --timeout 300 --timeout-method thread \
  -k "nodes or level_kernel_equals or 2perstage_nodes" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python tools/bench_sc.py --scenario 2perstage --kernel all --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']; print(d['config']['kernel'], round(r['avg_kernel_us'],1), 'us', round(r['frac'],3), '%.3e'%d['value'])"
