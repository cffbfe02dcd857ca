cd "${GRAFT_REPO_ROOT:-/root/repo}"
for mb in 0 256 384 512 128; do
  for v in base nodma; do
    root=gym-supplychain_amd; [ $v != base ] && root=exp/$v
    SCG_PKG_ROOT=$root timeout -k 10 200 python tools/bench_sc.py --no-cpu-baseline --scenario 2perstage --kernel nodes --steps 100 --nodes-max-blocks $mb > gpurun_out/mb_${v}_$mb.log 2>&1 || exit 1
    echo -n "mb $mb $v "; grep '^{' gpurun_out/mb_${v}_$mb.log | python -c "
import json,sys
for l in sys.stdin:
  d=json.loads(l); print('kern_us %.2f'%d['roofline']['avg_kernel_us'])"
  done
done
