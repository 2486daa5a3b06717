#!/bin/bash
# Round 5 (am): kernel traces of the C4 and C5 lines on the current tree (per-kernel durations and gaps of a frame)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for cfg in C4 C5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05am_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 40 --warmup 10 $common > gpurun_out/r05am_$cfg.log 2>&1 || { tail -5 gpurun_out/r05am_$cfg.log; exit 1; }
  python3 scripts/trace_summary.py gpurun_out/r05am_$cfg 10 > gpurun_out/r05am_${cfg}_summary.txt 2>&1
  cat gpurun_out/r05am_${cfg}_summary.txt
done
