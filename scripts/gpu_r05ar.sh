#!/bin/bash
# Round 5 (ar): the inter-frame idle gap of the two-launch frames (C5) with the bench's event brackets off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0 --no-timing"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05ar_C5 -o run --output-format csv -- python3 bench.py --config C5 --steps 40 --warmup 10 $common > gpurun_out/r05ar_C5.log 2>&1 || { tail -5 gpurun_out/r05ar_C5.log; exit 1; }
python3 scripts/trace_summary.py gpurun_out/r05ar_C5 12 > gpurun_out/r05ar_C5_summary.txt 2>&1
cat gpurun_out/r05ar_C5_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05ar_C2 -o run --output-format csv -- python3 bench.py --steps 40 --warmup 10 $common > gpurun_out/r05ar_C2.log 2>&1 || { tail -5 gpurun_out/r05ar_C2.log; exit 1; }
python3 scripts/trace_summary.py gpurun_out/r05ar_C2 6 > gpurun_out/r05ar_C2_summary.txt 2>&1
cat gpurun_out/r05ar_C2_summary.txt
