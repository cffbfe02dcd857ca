cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/stampexp; mkdir -p $OUT
for rep in 1 2 3 4; do
for v in "st:" "un:--unstamped-headline"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 $a --no-cpu-baseline --no-extras --kernel-samples 35 > $OUT/$name$rep.log 2>&1 || { echo "$name failed"; tail -5 $OUT/$name$rep.log; exit 1; }
  grep '^{' $OUT/$name$rep.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']
print('$name', '%.3e'%d['value'], round(d['ms_per_step']*1e3,2),'us/step', round(r['avg_kernel_us'],2))"
done; done
