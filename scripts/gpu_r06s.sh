#!/bin/bash
# Round 6 (s): k_weigh_pk12 tuning sweep at C3 (marker phase width 2 / 3 / 4 (tree) / 6, no sched_barrier between
# phases, a 2-wave occupancy floor), ab/libpfmpe_<variant>.so built by scripts/build_variant.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
  for v in tree ph3 ph6 ph2 nofence w2; do
    if [ $v = tree ]; then unset PFMPE_LIB_OVERRIDE; else export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_$v.so; fi
    timeout -k 10 200 python -u bench.py --config C3 --steps 300 --warmup 10 $common > gpurun_out/r06/ab_s_$v.log 2>&1 || { tail -5 gpurun_out/r06/ab_s_$v.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06/ab_s_$v.log').read().splitlines() if l.startswith('{')][-1])
r=d['roofline']; print('C3 $v', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,2), 'G', r['per_kernel_avg_us'])" | tee -a gpurun_out/r06/ab_s.txt
  done
done
unset PFMPE_LIB_OVERRIDE
