#!/bin/bash
# One GPU-box session: GPU tests, smoke, short bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/timeout (rc not in {0,1}) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name" ; date
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
what=${1:-all}
if [ "$what" = all ] || [ "$what" = tests ]; then
  step pytest_gpu 700 python -m pytest tests -m gpu -q -rf --timeout=600 || true
fi
if [ "$what" = all ] || [ "$what" = smoke ]; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
if [ "$what" = all ] || [ "$what" = bench ]; then
  step bench 600 python bench.py --steps 200 --warmup 20 || exit 1
fi
if [ "$what" = all ] || [ "$what" = prof ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --cpu-frames 0 --no-timing || exit 1
fi
if [ "$what" = all ] || [ "$what" = bench ]; then
  step bench_pyloop 600 python bench.py --steps 200 --warmup 20 --cpu-frames 0 --python-loop || exit 1
fi
if [ "$what" = all ] || [ "$what" = pmc ]; then
  step pmc 1000 bash scripts/pmc.sh c2_n100000 --steps 100 --warmup 10 || exit 1
fi
echo done
