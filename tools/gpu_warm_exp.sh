cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/warm2; mkdir -p $OUT
for rep in 1 2 3 4; do
for v in "base:--warmup 5" "dry:--warmup 5 --dry-region 1" "dryspin:--warmup 5 --dry-region 1 --spin" "w350dry:--warmup 350 --dry-region 1"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 120 python bench.py --steps 20 $a --no-cpu-baseline --no-extras --kernel-samples 35 > $OUT/$name$rep.log 2>&1 || { echo "$name failed"; tail -5 $OUT/$name$rep.log; exit 1; }
  grep '^{' $OUT/$name$rep.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']
print('$name', d['warmup_steps_run'], '%.3e'%d['value'], round(d['ms_per_step']*1e3,2),'us/step', round(r['avg_kernel_us'],2), 'span', round(r['isolated_kernel_us'],2),'iso', '%.3e'%d['episodes_timed']['value'])"
done; done
