#!/bin/bash
# Round 5 (as): kernel trace of the 2 x C4 batch (pfmpe_step_multi) beside the one-stream C4 frames
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
common="--cpu-frames 0 --worst-frames 0 --single-points none --scale-ref-steps 0 --exact-steps 0 --no-timing"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r05as -o run --output-format csv -- python3 bench.py --config C4 --steps 20 --warmup 5 --multi-sweep 2 --multi-groups 1 --multi-steps 60 $common > gpurun_out/r05as.log 2>&1 || { tail -5 gpurun_out/r05as.log; exit 1; }
python3 scripts/trace_summary.py gpurun_out/r05as 14 > gpurun_out/r05as_summary.txt 2>&1
cat gpurun_out/r05as_summary.txt
timeout -k 10 300 python -u scripts/diag_multi_host.py --config C4 --S 2 --steps 30 > gpurun_out/r05as_host.txt 2>&1; cat gpurun_out/r05as_host.txt
