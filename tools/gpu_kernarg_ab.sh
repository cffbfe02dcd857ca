#!/bin/bash
# The driver's bench configuration (--steps 20 --warmup 5) under HIP runtime kernarg settings,
# interleaved, 3 rounds, one box (host enqueue vs GPU time of a short region).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
declare -A CFG=( [default]="" [devka0]="HIP_FORCE_DEV_KERNARG=0" [devka1]="HIP_FORCE_DEV_KERNARG=1"
                 [hdp0]="DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0" [fgs1]="ROC_USE_FGS_KERNARG=1" [copyopt0]="DEBUG_HIP_KERNARG_COPY_OPT=0" )
for r in 1 2 3; do
  for c in default devka0 devka1 hdp0 fgs1 copyopt0; do
    env ${CFG[$c]} timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/ka_${c}_$r.log 2>&1 || { echo "FAIL $c"; tail -3 gpurun_out/ka_${c}_$r.log; exit 1; }
    echo -n "== $r $c "; grep '^{' gpurun_out/ka_${c}_$r.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); h=d.get('headline_split',{})
print('value %.3e ms/step %.2f us kern %.2f enq %s'%(d['value'], d['ms_per_step']*1e3, d['roofline']['avg_kernel_us'], h.get('enqueue_us_per_step')))"
  done
done
