#!/bin/bash
# Round 5 (ab): resident frame time vs run length (is a long dispatch slower?)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0 --no-timing"
for st in 30 100 200 1000; do
  for res in 1 0; do
    timeout -k 10 200 python -u bench.py --resident $res --steps $st --warmup 10 $common > gpurun_out/r05ab_b.log 2>&1 || { tail -5 gpurun_out/r05ab_b.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r05ab_b.log').read().strip().splitlines()[-1])
print('steps=$st resident=$res', round(d['ms_per_step']*1e3,2), 'us/frame')" | tee -a gpurun_out/r05ab_ab.txt
  done
done
