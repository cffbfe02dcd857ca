#!/bin/bash
# Each SupplyChain kernel on sc-2perstage-v0 (65,536 envs), with and without build_info ledgers
# (is another kernel a better ledger path than the node-parallel one?).  tools/gpu_kernel_ledgers.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
for k in lane staged nodes; do
  for bi in "" "--build-info"; do
    timeout -k 10 200 python tools/bench_sc.py --no-cpu-baseline --scenario 2perstage --kernel $k --steps 100 $bi > gpurun_out/kled_r05t_${k}${bi}.log 2>&1 || { echo "FAIL $k $bi"; tail -5 gpurun_out/kled_r05t_${k}${bi}.log; exit 1; }
    echo -n "== $k $bi "; grep '^{' gpurun_out/kled_r05t_${k}${bi}.log | python -c "
import json,sys
for l in sys.stdin:
  d=json.loads(l); print(d['config']['kernel'], 'kern_us %.2f'%d['roofline']['avg_kernel_us'])"
  done
done
