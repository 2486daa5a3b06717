#!/bin/bash
# Round 6 (w): the dispatch form. Every kernel as hipExtLaunchKernel with a (never read) stop event
# (PFMPE_DIAG 524288) vs plain hipLaunchKernel: the trace showed the two-launch frames' kernels 4-13 % shorter in
# the event-carrying kernel pass than back to back in the timed region.  C4 / C3 / C5 / C2 frames, two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
for cfg in C4 C3 C5 C2; do
  for d in 524288 0; do
    timeout -k 10 200 python -u bench.py --config $cfg --steps 300 --warmup 10 --diag $d $common > gpurun_out/r06/ab_w_$d.log 2>&1 || { tail -5 gpurun_out/r06/ab_w_$d.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06/ab_w_$d.log').read().splitlines() if l.startswith('{')][-1])
r=d['roofline']; print('$cfg diag $d', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,2), 'G', r['per_kernel_avg_us'])" | tee -a gpurun_out/r06/ab_w.txt
  done
done
done
