#!/bin/bash
# tools/bench_sc.py kernel time per exp/ variant, alternated REPS times (no tests, no CPU
# baseline): gpu_sc_var_ab.sh OUT_LOG SCENARIO "V1 V2 ..." [extra bench_sc args]
set -o pipefail
out=$1; scen=$2; vars=$3; shift 3
echo "# bench_sc --scenario $scen $* per variant ($vars), ${REPS:-3} alternations" > "$out"
for rep in $(seq 1 ${REPS:-3}); do
  for v in $vars; do
    SCG_PKG_ROOT=exp/$v timeout -k 10 240 python -u tools/bench_sc.py --no-cpu-baseline --scenario $scen "$@" > /tmp/scab.log 2>&1 || { cat /tmp/scab.log >> "$out"; exit 1; }
    grep '^{' /tmp/scab.log | python -c "
import json,sys
for l in sys.stdin:
  d=json.loads(l); r=d['roofline']
  print('$v', $rep, d['config']['workload'][:24], d['config'].get('n_envs'), 'kern_us %.2f' % r['avg_kernel_us'], 'frac %.3f' % r['frac'])" >> "$out"
  done
done
