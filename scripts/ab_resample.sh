#!/bin/bash
# The streaming resampling pass: its bit-identity test, then an alternating A/B (default vs
# --diag 2048 = one block per 256 particles) at C4 / C3 / C5.  Every GPU step is time-limited; stop on failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
t=${TAG:-abr}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_frame_shapes.py \
  -k "streaming_resampling or kept_propagated or c4_full" > gpurun_out/${t}_tests.log 2>&1 || { tail -30 gpurun_out/${t}_tests.log; exit 1; }
tail -3 gpurun_out/${t}_tests.log
for r in 1 2; do
  for cfg in ${AB_CFGS:-C4 C3 C5}; do
    for d in 0 2048; do
      timeout -k 10 200 python bench.py --config $cfg --cpu-frames 0 --worst-frames 0 --steps 60 --warmup 6 --diag $d \
        > gpurun_out/${t}_${cfg}_$d.log 2>&1 || { tail gpurun_out/${t}_${cfg}_$d.log; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/${t}_${cfg}_$d.log')); print('$cfg diag $d', round(d['ms_per_step']*1e3,2), 'us/frame', d['roofline']['per_kernel_avg_us'])"
    done
  done
done
