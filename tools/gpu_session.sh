#!/bin/bash
# One GPU session on the box (run through gpurun): parity tests, smoke, the bench (default
# and the driver's configuration), the SupplyChain bench with its same-host CPU baseline,
# rocprofv3 kernel stats of the bench, and HBM traffic (FETCH_SIZE and WRITE_SIZE, one pass
# each) of the BeerGame step kernel and of each SupplyChain scenario's auto kernel. Every GPU
# step has its own time limit; any failure stops the script.
#   tools/gpu_session.sh TAG [STEPS]
#   STEPS: comma list of tests,smoke,bench,pg,sc,led,sweep,prof,pmc,scpmc (default all)
#   pg: bench.py at one rank under torch.distributed.run with SCG_BENCH_PG=1 (the RCCL group,
#   node barrier and return all-gather of the multi-GPU flow)
# PMC summaries (here, after the pull):
#   python tools/pmc_summary.py gpurun_out/pmc_TAG --meta bench=beergame-v0 n_envs=65536 --family bg
#   python tools/pmc_summary.py gpurun_out/scpmc_TAG/SCN --meta bench=bench_sc scenario=SCN n_envs=N \
#       kernel=auto build_info=false --family sc
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${1:-r04}
STEPS=",${2:-tests,smoke,bench,pg,sc,led,sweep,prof,pmc,scpmc},"
mkdir -p "$OUT"
stop() { echo "step '$1' ended with $2: stopping"; exit "$2"; }
want() { [[ "$STEPS" == *",$1,"* ]]; }
run() {  # run NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -v amdgpu.ids "$OUT/${name}_$TAG.log" | tail -3 | cut -c1-600
  [ $rc -ne 0 ] && stop "$name" $rc
  return 0
}
srchash() { python3 -c "import sys; sys.path.insert(0, '$ROOT'); import bench; print(bench.kernel_sources_hash('$1'))"; }
want tests && run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
want smoke && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
want bench && run bench 400 python bench.py
want bench && run bench_driver 300 python bench.py --steps 20 --warmup 5
want pg && run bench_pg 300 env SCG_BENCH_PG=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
want sc && run bench_sc 900 python tools/bench_sc.py --scenario all --kernel auto
want led && run bench_sc_ledgers 600 python tools/bench_sc.py --scenario both --kernel auto --build-info --no-cpu-baseline
want sweep && run sweep_bg 600 python tools/sweep_bg.py --max-log2 24
cd /tmp && export TMPDIR=/tmp
if want prof; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o bench -- \
      python3 "$ROOT/bench.py" --no-cpu-baseline --no-extras > "$OUT/prof_$TAG.log" 2>&1
  rc=$?; echo "rocprofv3 rc=$rc"; [ $rc -ne 0 ] && stop rocprof $rc
fi
if want pmc; then
  PM=$OUT/pmc_$TAG; mkdir -p "$PM"; srchash bg > "$PM/src_hash_bg.txt"
  BG="python3 $ROOT/bench.py --no-cpu-baseline --no-extras --steps 700 --warmup 70"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$PM/bg_fetch" -o pmc -- $BG > "$PM/bg_fetch.log" 2>&1 || stop pmc_fetch $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$PM/bg_write" -o pmc -- $BG > "$PM/bg_write.log" 2>&1 || stop pmc_write $?
  echo "pmc ok"
fi
if want scpmc; then
  for scn in 2perstage 2perstage_mp ntom; do
    PM=$OUT/scpmc_$TAG/$scn; mkdir -p "$PM"; srchash sc > "$PM/src_hash_sc.txt"
    SC="python3 $ROOT/tools/bench_sc.py --no-cpu-baseline --steps 6 --warmup 1 --scenario $scn --kernel auto"
    timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$PM/sc_fetch" -o pmc -- $SC > "$PM/sc_fetch.log" 2>&1 || stop "scpmc_fetch_$scn" $?
    timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$PM/sc_write" -o pmc -- $SC > "$PM/sc_write.log" 2>&1 || stop "scpmc_write_$scn" $?
  done
  echo "scpmc ok"
fi
exit 0
