#!/bin/bash
# The default C2 line under the driver's flags (--steps 20 --warmup 5) with the dispatch-event sampling period
# varied (1, 2 = the default at 20 steps, 5, 20, none) and with a longer warmup, two rounds, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
COMMON="--cpu-frames 0 --worst-frames 0 --multi-sweep none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
  for v in "--timing-period 1" "--timing-period 2" "--timing-period 5" "--timing-period 20" "--no-timing" "--warmup 100 --timing-period 5"; do
    timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 $COMMON $v > gpurun_out/bt.log 2>&1 || { tail -3 gpurun_out/bt.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/bt.log').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[1].ljust(32), round(d['ms_per_step']*1e3,2), 'us/frame', r.get('avg_us'), r.get('launches_timed'))" "$v"
  done
done
