#!/bin/bash
# Round 4 closing pass: the whole GPU suite, smoke(), the driver's own bench command and its kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r04e_suite.log 2>&1; r=$?
tail -5 gpurun_out/r04e_suite.log
[ $r -eq 0 ] || exit $r
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04e_smoke.log 2>&1 \
  || { tail -5 gpurun_out/r04e_smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04e_bench_driver.log 2>&1 \
  || { tail -5 gpurun_out/r04e_bench_driver.log; exit 1; }
tail -c 3000 gpurun_out/r04e_bench_driver.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04e_trace -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04e_trace.log 2>&1 || { tail -5 gpurun_out/r04e_trace.log; exit 1; }
f=$(find gpurun_out/r04e_trace -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -c1-160 "$f"
