cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_cas.log 2>&1; rc=$?; tail -2 gpurun_out/pt_cas.log; [ $rc -ne 0 ] && exit $rc
for v in base old; do
  root=gym-supplychain_amd; [ $v != base ] && root=exp/$v
  SCG_PKG_ROOT=$root timeout -k 10 300 python tools/bench_sc.py --no-cpu-baseline --kernel all > gpurun_out/sc_cas_$v.log 2>&1 || exit 1
  echo "== $v"; grep '^{' gpurun_out/sc_cas_$v.log | python -c "
import json,sys
for l in sys.stdin:
  d=json.loads(l); print(d['config']['workload'][:22], d['config']['kernel'], '%.3e'%d['value'], 'kern_us %.1f'%d['roofline']['avg_kernel_us'], 'frac %.3f'%d['roofline']['frac'])"
done
