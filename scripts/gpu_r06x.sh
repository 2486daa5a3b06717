#!/bin/bash
# Round 6 (x): k_resample_owners occupancy floor 4 / 5 / 8 waves per SIMD against the tree's 6 (ab/libpfmpe_ow*.so;
# base = the tree's library), C4 / C5 / C3, two rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
for cfg in C4 C5 C3; do
  for v in base ow4 ow5 ow8; do
    export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_$v.so
    timeout -k 10 200 python -u bench.py --config $cfg --steps 300 --warmup 10 $common > gpurun_out/r06/ab_x_$v.log 2>&1 || { tail -5 gpurun_out/r06/ab_x_$v.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06/ab_x_$v.log').read().splitlines() if l.startswith('{')][-1])
r=d['roofline']; print('$cfg $v', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,2), 'G', r['per_kernel_avg_us'])" | tee -a gpurun_out/r06/ab_x.txt
  done
done
done
unset PFMPE_LIB_OVERRIDE
