#!/bin/bash
# One GPU session on the box (run through gpurun): parity tests, smoke, the bench (default
# and the driver's configuration), the SupplyChain bench, rocprofv3 kernel stats of the
# bench, and the BeerGame step kernel's HBM traffic (FETCH_SIZE and WRITE_SIZE, one pass
# each). Every GPU step has its own time limit; any failure stops the script.
#   tools/gpu_session.sh TAG [STEPS]     STEPS: comma list of tests,smoke,bench,sc,prof,pmc (default all)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${1:-r03}
STEPS=",${2:-tests,smoke,bench,sc,prof,pmc},"
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
want tests && run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
want smoke && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
want bench && run bench 400 python bench.py
want bench && run bench_driver 300 python bench.py --steps 20 --warmup 5
want sc && run bench_sc 600 python tools/bench_sc.py --kernel both --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
if want prof; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o bench -- \
      python3 "$ROOT/bench.py" --no-cpu-baseline --no-extras > "$OUT/prof_$TAG.log" 2>&1
  rc=$?; echo "rocprofv3 rc=$rc"; [ $rc -ne 0 ] && stop rocprof $rc
fi
if want pmc; then
  PM=$OUT/pmc_$TAG; mkdir -p "$PM"
  BG="python3 $ROOT/bench.py --no-cpu-baseline --no-extras --steps 700 --warmup 70"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$PM/bg_fetch" -o pmc -- $BG > "$PM/bg_fetch.log" 2>&1 || stop pmc_fetch $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$PM/bg_write" -o pmc -- $BG > "$PM/bg_write.log" 2>&1 || stop pmc_write $?
  echo "pmc ok"
fi
exit 0
