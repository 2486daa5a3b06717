#!/bin/bash
# Round 5 (aa): C2 resident vs launched after the start-up change, C loop and python loop
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
  for res in 1 0; do
    for pl in "" "--python-loop"; do
      timeout -k 10 200 python -u bench.py --resident $res $pl --steps 2000 --warmup 50 $common > gpurun_out/r05aa_b.log 2>&1 || { tail -5 gpurun_out/r05aa_b.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('gpurun_out/r05aa_b.log').read().strip().splitlines()[-1])
r=d.get('roofline') or {}
print('resident=$res $pl', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,3), 'G', r.get('kernel'), r.get('avg_us'))" | tee -a gpurun_out/r05aa_ab.txt
    done
  done
done
