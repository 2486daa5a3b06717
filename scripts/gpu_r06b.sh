#!/bin/bash
# Round 6 (b): the whole -m gpu suite on the tree without the resident server and with the fused owners finish,
# then the driver's bench command, its kernel trace and the trace check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/gpu_suite_b.log 2>&1; r=$?
tail -n 30 gpurun_out/r06/gpu_suite_b.log | grep -v "^$" | tail -12
[ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/bench_driver_b.log 2>&1 || { tail -20 gpurun_out/r06/bench_driver_b.log; exit 1; }
tail -c 1500 gpurun_out/r06/bench_driver_b.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/trace_b -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/trace_b.log 2>&1 || { tail -20 gpurun_out/r06/trace_b.log; exit 1; }
d=$(dirname $(find gpurun_out/r06/trace_b -name run_kernel_trace.csv | head -1))
python3 scripts/trace_check.py $d gpurun_out/r06/trace_b.log | tee gpurun_out/r06/trace_check_b.txt
python3 scripts/trace_summary.py $d 12 > gpurun_out/r06/trace_summary_b.txt
