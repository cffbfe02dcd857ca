#!/bin/bash
# Host-side cost of a step and the driver-config bench, three times each.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=${1:-host}
O=gpurun_out/host_$TAG.log
: > $O
for i in 1 2 3; do
  timeout -k 10 120 python tools/host_overhead.py >> $O 2>&1 || exit $?
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras >> $O 2>&1 || exit $?
done
grep -v amdgpu.ids $O | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l)
    if 'metric' in d: print('bench value %.3e ms_per_step %.4f kernel %.3f ep_value %.3e ep_kernel %.3f' % (d['value'], d['ms_per_step']*1e3, d['roofline']['avg_kernel_us'], d['episodes_timed']['value'], d['episodes_timed']['avg_kernel_us']))
    else: print('host', {k: round(v,3) for k,v in d.items() if isinstance(v,float)})
"
