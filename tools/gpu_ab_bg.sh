#!/bin/bash
# A/B of BeerGame step-kernel builds on one box: exp/<name> variants (tools/exp_build.py)
# against the working tree, interleaved twice. Then the GPU tests.
#   tools/gpu_ab_bg.sh TAG VARIANT...
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=$1; shift
O=gpurun_out/ab_$TAG.log
: > $O
for rep in 1 2; do
  for v in "$@" tree; do
    if [ $v = tree ]; then P=""; else P="exp/$v"; fi
    SCG_PKG_ROOT=$P timeout -k 10 120 python tools/bg_ab.py --label $v >> $O 2>&1 || exit $?
  done
done
grep label $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_$TAG.log
exit $rc
