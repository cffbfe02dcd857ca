#!/bin/bash
# bench.py in the driver's configuration under HIP runtime environment variants, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/envexp_$1; mkdir -p $OUT
for rep in 1 2 3 4; do
for v in "dflt:" "dk0:HIP_FORCE_DEV_KERNARG=0" "dk1:HIP_FORCE_DEV_KERNARG=1"; do
  name=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --kernel-samples 35 > $OUT/$name$rep.log 2>&1 || { echo "$name failed"; tail -5 $OUT/$name$rep.log; exit 1; }
  grep '^{' $OUT/$name$rep.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']
print('$name', '%.3e'%d['value'], round(d['ms_per_step']*1e3,2),'us/step', round(r['avg_kernel_us'],2), 'ep %.3e'%d['episodes_timed']['value'], 'iso', round(r['isolated_kernel_us'],2))"
done; done
