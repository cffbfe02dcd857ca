cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/warm3; mkdir -p $OUT
for rep in 1 2 3; do
for v in "m5:5" "m35:35" "m175:175" "m700:700"; do
  name=${v%%:*}; m=${v#*:}
  SCG_BENCH_MIN_WARMUP=$m timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --kernel-samples 35 > $OUT/$name$rep.log 2>&1 || { echo "$name failed"; tail -5 $OUT/$name$rep.log; exit 1; }
  grep '^{' $OUT/$name$rep.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']
print('$name', d['warmup_steps_run'], '%.3e'%d['value'], round(d['ms_per_step']*1e3,2),'us/step', round(r['avg_kernel_us'],2))"
done; done
