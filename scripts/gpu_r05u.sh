#!/bin/bash
# Round 5 (u): kernel traces of one C4 stream and of the 2 x C4 batch (batch >= single)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
common="--cpu-frames 0 --worst-frames 0 --single-points none --scale-ref-steps 0 --exact-steps 0 --no-timing"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05u_single -o run --output-format csv -- python3 bench.py --config C4 --steps 60 --warmup 10 --multi-sweep none $common > gpurun_out/r05u_single.log 2>&1 || { tail gpurun_out/r05u_single.log; exit 1; }
python3 scripts/trace_summary.py gpurun_out/r05u_single/*/ 2>/dev/null | head -12 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05u_multi -o run --output-format csv -- python3 bench.py --config C4 --steps 3 --warmup 1 --multi-sweep 2 --multi-groups 1 --multi-steps 30 $common > gpurun_out/r05u_multi.log 2>&1 || { tail gpurun_out/r05u_multi.log; exit 1; }
tail -c 400 gpurun_out/r05u_multi.log
