#!/bin/bash
# N-sweep of the SupplyChain auto kernels on the final tree: sc-2perstage (node-parallel) at
# 16,384 .. 1,048,576 envs and ntom (staged) at 65,536 .. 524,288 envs, one line per size.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/sc_nsweep_${1:-r05}.log; : > $OUT
for n in 16384 32768 65536 131072 262144 524288 1048576; do
  timeout -k 10 200 python tools/bench_sc.py --no-cpu-baseline --scenario 2perstage --envs $n --steps 50 >> $OUT 2>&1 || exit 1
done
for n in 65536 131072 262144 524288; do
  timeout -k 10 300 python tools/bench_sc.py --no-cpu-baseline --scenario ntom --envs $n --steps 20 >> $OUT 2>&1 || exit 1
done
grep '^{' $OUT | python -c "
import json,sys
for l in sys.stdin:
  d=json.loads(l); r=d['roofline']
  print(d['config']['workload'][:24], d['config']['n_envs'], d['config']['kernel'], 'kern_us %.2f'%r['avg_kernel_us'], 'frac %.3f'%r['frac'], 'envsteps/s %.3e'%d['value'])"
