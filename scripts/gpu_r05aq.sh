#!/bin/bash
# Round 5 (ah): C2 2,000-frame A/B of the integer-key group argmax (new) against the previous build, three alternating rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2 3; do
  for v in new base; do
    if [ $v = base ]; then export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_base.so; else unset PFMPE_LIB_OVERRIDE; fi
    timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 $common > gpurun_out/r05aq_b_$v.log 2>&1 || { tail -5 gpurun_out/r05aq_b_$v.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r05aq_b_$v.log').read().strip().splitlines()[-1])
r=d.get('roofline') or {}
print('$v', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,3), 'G', r.get('kernel'), r.get('avg_us'))" | tee -a gpurun_out/r05aq_ab.txt
  done
done
