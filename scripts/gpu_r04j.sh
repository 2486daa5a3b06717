#!/bin/bash
# Round 4: the batched and hand-off kernels after the map-staging and k_top_wide changes (identity tests), then the
# C2 driver-setting frame with four bracketed frames, and the 2 x C4 / 32 x C5 batches with their kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_frame_shapes.py tests/test_gpu_defer.py -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04j_tests.log 2>&1 || { tail -20 gpurun_out/r04j_tests.log; exit 1; }
tail -2 gpurun_out/r04j_tests.log
for rep in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-frames 0 --worst-frames 0 --scale-ref-steps 0 \
    --exact-steps 0 --multi-sweep none --single-points none > gpurun_out/r04j_drv_$rep.log 2>&1 || { tail -5 gpurun_out/r04j_drv_$rep.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04j_drv_$rep.log').read().strip().splitlines()[-1])
print('drv', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,3), 'G/s', d['roofline']['per_kernel_avg_us'], d['roofline']['launches_timed'])"
done
timeout -k 10 300 python -u bench.py --config C4 --steps 20 --warmup 5 --cpu-frames 0 --worst-frames 0 \
  --multi-sweep 2 --multi-groups 1 --multi-steps 30 --single-points none > gpurun_out/r04j_c4.log 2>&1 || { tail -5 gpurun_out/r04j_c4.log; exit 1; }
timeout -k 10 300 python -u bench.py --config C5 --steps 20 --warmup 5 --cpu-frames 0 --worst-frames 0 \
  --multi-sweep 32 --multi-groups 2 --multi-steps 30 --single-points none > gpurun_out/r04j_c5.log 2>&1 || { tail -5 gpurun_out/r04j_c5.log; exit 1; }
for c in c4 c5; do python3 -c "
import json; d=json.loads(open('gpurun_out/r04j_$c.log').read().strip().splitlines()[-1])
print('$c single', round(d['ms_per_step']*1e3,1), 'us', round(d['value']/1e9,2), 'G/s', d['roofline']['per_kernel_avg_us'], '|',
      [(p['streams'], p['groups'], round(p['updates_per_s']/1e9,2), p['frac'], round(p['ms_per_batch']*1e3,1)) for p in d['multi_stream']['points']])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04j_c4x2 -o run -- python3 bench.py \
  --config C4 --steps 5 --warmup 2 --cpu-frames 0 --worst-frames 0 --multi-sweep 2 --multi-groups 1 --multi-steps 20 \
  --no-timing --single-points none > gpurun_out/r04j_c4x2.log 2>&1 || { tail -5 gpurun_out/r04j_c4x2.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r04j_c4x2/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:60]:60s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:9.2f} us")
PY
