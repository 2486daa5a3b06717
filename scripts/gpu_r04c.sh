#!/bin/bash
# Round 4, the C2 (k_frame2) latency chain: a fresh phase-stamp timeline, the driver's own bench settings
# (--steps 20 --warmup 5) with and without HIP-event brackets in the timed region, and the kernel trace of that
# command.  Logs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/diag_stamps.py 100000 > gpurun_out/r04c_stamps_c2.log 2>&1 \
  || { tail -5 gpurun_out/r04c_stamps_c2.log; exit 1; }
cat gpurun_out/r04c_stamps_c2.log
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --cpu-frames 0 --worst-frames 0 --scale-ref-steps 0 --exact-steps 0 \
    --multi-sweep none --single-points none "$@" > gpurun_out/r04c_$tag.log 2>&1 || { tail -5 gpurun_out/r04c_$tag.log; return 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04c_$tag.log').read().strip().splitlines()[-1])
r=d['roofline'] or {}
print('$tag', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,3), 'G/s', r.get('per_kernel_avg_us'), r.get('launches_timed'))"
}
for rep in 1 2 3; do
  run drv_$rep --steps 20 --warmup 5 || exit 1
  run drv_notiming_$rep --steps 20 --warmup 5 --no-timing || exit 1
  run drv_p10_$rep --steps 20 --warmup 5 --timing-period 10 || exit 1
  run long_$rep --steps 200 --warmup 20 || exit 1
  HIP_FORCE_DEV_KERNARG=1 run devka_$rep --steps 20 --warmup 5 || exit 1
  HIP_FORCE_DEV_KERNARG=0 run hostka_$rep --steps 20 --warmup 5 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04c_trace -o run -- \
  python3 bench.py --steps 20 --warmup 5 --cpu-frames 0 --worst-frames 0 --scale-ref-steps 0 --exact-steps 0 \
  --multi-sweep none --single-points none > gpurun_out/r04c_trace.log 2>&1 || { tail -5 gpurun_out/r04c_trace.log; exit 1; }
f=$(find gpurun_out/r04c_trace -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cat "$f"
