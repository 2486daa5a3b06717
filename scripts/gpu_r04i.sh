#!/bin/bash
# Round 4: C2 at the driver's settings after the timing-event preallocation and the time-based stream query; the
# default bench line (with the C3 / C4 single-stream points); a kernel trace of the 2 x C4 batch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --cpu-frames 0 --worst-frames 0 --scale-ref-steps 0 --exact-steps 0 \
    --multi-sweep none --single-points none "$@" > gpurun_out/r04i_$tag.log 2>&1 || { tail -5 gpurun_out/r04i_$tag.log; return 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04i_$tag.log').read().strip().splitlines()[-1])
r=d['roofline'] or {}
print('$tag', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,3), 'G/s', r.get('per_kernel_avg_us'), r.get('launches_timed'))"
}
for rep in 1 2 3; do
  run drv_$rep --steps 20 --warmup 5 || exit 1
  run drv_notiming_$rep --steps 20 --warmup 5 --no-timing || exit 1
  run long_$rep --steps 200 --warmup 20 || exit 1
done
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04i_default.log 2>&1 || { tail -5 gpurun_out/r04i_default.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04i_default.log').read().strip().splitlines()[-1])
print('default', round(d['ms_per_step']*1e3,2), 'us', round(d['value']/1e9,3), 'G', d['roofline']['frac'], d['roofline']['per_kernel_avg_us'])
for k, v in (d.get('single_stream') or {}).items(): print(k, v)
print([(p['config'], p['streams'], p['groups'], round(p['updates_per_s']/1e9,2), p['frac']) for p in d['multi_stream']['points']])
print('scale_ref', d['scaling_reference']); print('parity', d['parity_mode']); print('worst', d['worst_case']); print('cpu', d['cpu_baseline'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04i_c4x2 -o run -- python3 bench.py \
  --config C4 --steps 5 --warmup 2 --cpu-frames 0 --worst-frames 0 --multi-sweep 2 --multi-groups 1 --multi-steps 20 \
  --no-timing > gpurun_out/r04i_c4x2.log 2>&1 || { tail -5 gpurun_out/r04i_c4x2.log; exit 1; }
f=$(find gpurun_out/r04i_c4x2 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -c1-120 "$f" | awk -F, '{print $1, $2, $4}'
