#!/bin/bash
# Round 5 (y): the driver's default bench command, then the kernel trace of the C2 line (same steps) for profiles/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > gpurun_out/r05y_bench.log 2>&1 || { tail -5 gpurun_out/r05y_bench.log; exit 1; }
tail -c 300 gpurun_out/r05y_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05y_prof -o run --output-format csv -- python3 bench.py --cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0 > gpurun_out/r05y_prof.log 2>&1 || { tail -5 gpurun_out/r05y_prof.log; exit 1; }
python3 scripts/trace_summary.py gpurun_out/r05y_prof 6 > gpurun_out/r05y_trace_summary.txt 2>&1; head -5 gpurun_out/r05y_trace_summary.txt
