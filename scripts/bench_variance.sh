#!/bin/bash
# Default C2 line under the driver's flags (--steps 20 --warmup 5) with and without the sampled dispatch
# events, and at the bench defaults, alternating; one JSON summary line per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
COMMON="--cpu-frames 0 --worst-frames 0 --multi-sweep none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
  for v in "--steps 20 --warmup 5" "--steps 20 --warmup 5 --no-timing" "--steps 200 --warmup 20"; do
    timeout -k 10 120 python -u bench.py $v $COMMON > gpurun_out/bv.log 2>&1 || { tail gpurun_out/bv.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/bv.log').read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step']*1e3,2), 'us/frame', d['roofline'].get('avg_us'))" "$v"
  done
done
