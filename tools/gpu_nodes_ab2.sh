#!/bin/bash
# node-parallel kernel parity tests on the tree, then an A/B against exp/ variants.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/nodes_$1; shift; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_supplychain.py -x -q --timeout 300 --timeout-method thread \
  -k "nodes or level_kernel_equals or auto_kernel" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/gpu_nodes_ab.sh ab_$(basename $OUT) "$@"
