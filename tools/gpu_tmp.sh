SC_NO_PMC=1 bash tools/gpu_sc_ab.sh f chunk8 chunk16
cd gpurun_out/sc_f && for f in bench_*.log; do echo "$f"; grep '^{' $f | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('   ', d['config']['kernel'], d['config']['n_envs'], round(d['roofline']['avg_kernel_us'],1), 'us', round(d['roofline']['frac'],3))"; done
