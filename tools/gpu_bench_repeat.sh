#!/bin/bash
# Repeated bench.py runs on one box: 3 with the defaults, 5 in the driver's configuration.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/rep_$1; mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/default$i.log 2>&1 || { tail -5 $OUT/default$i.log; exit 1; }
done
for i in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/driver$i.log 2>&1 || { tail -5 $OUT/driver$i.log; exit 1; }
done
for f in $OUT/*.log; do grep '^{' $f | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']
print('$(basename $f)', '%.3e'%d['value'], round(d['ms_per_step']*1e3,2),'us/step', round(r['avg_kernel_us'],2), 'us/launch', round(r['frac'],3))"; done
