#!/bin/bash
# Short-region variants (tools/short_region.py), interleaved twice.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=gpurun_out/short_$1.log
: > $O
for rep in 1 2; do
  timeout -k 10 120 python tools/short_region.py --label tree >> $O 2>&1 || exit $?
  timeout -k 10 120 python tools/short_region.py --label tree --spin >> $O 2>&1 || exit $?
  SCG_PKG_ROOT=exp/modlaunch timeout -k 10 120 python tools/short_region.py --label modlaunch >> $O 2>&1 || exit $?
  SCG_PKG_ROOT=exp/modlaunch timeout -k 10 120 python tools/short_region.py --label modlaunch --spin >> $O 2>&1 || exit $?
done
grep label $O
