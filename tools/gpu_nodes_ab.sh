#!/bin/bash
# sc-2perstage-v0 node-parallel kernel, tree and exp/ variants: tools/gpu_nodes_ab.sh TAG [VARIANT ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/nab_$1; shift; mkdir -p $OUT
for v in tree "$@"; do
  if [ "$v" = tree ]; then pk=""; else pk="$(pwd)/exp/$v"; fi
  SCG_BENCH_NO_CHECK=$NAB_NO_CHECK SCG_PKG_ROOT=$pk timeout -k 10 200 python tools/bench_sc.py --scenario 2perstage --kernel ${NAB_KERNEL:-nodes} --no-cpu-baseline --steps 60 > $OUT/$v.log 2>&1 || { echo "$v failed"; tail -5 $OUT/$v.log; exit 1; }
  grep '^{' $OUT/$v.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']; print('$v', d['config']['kernel'], round(r['avg_kernel_us'],1), 'us', round(r['frac'],3))"
done
