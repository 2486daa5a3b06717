#!/bin/bash
# Round 5 (q): k_frame2 / resident server with granule hand-offs: frame-shape + parity + resident tests, phases, C2 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_frame_shapes.py tests/test_gpu_resident.py tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/r05q_tests.log 2>&1 || { tail -40 gpurun_out/r05q_tests.log; exit 1; }
tail -n 1 gpurun_out/r05q_tests.log
timeout -k 10 200 python -u scripts/diag_resident.py > gpurun_out/r05q_diag.txt 2>&1 || { cat gpurun_out/r05q_diag.txt; exit 1; }
cat gpurun_out/r05q_diag.txt
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
  for res in 1 0; do
    timeout -k 10 200 python -u bench.py --resident $res --steps 2000 --warmup 50 $common > gpurun_out/r05q_b_${res}.log 2>&1 || { tail -5 gpurun_out/r05q_b_${res}.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r05q_b_${res}.log').read().strip().splitlines()[-1])
r=d.get('roofline') or {}
print('resident=$res', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,3), 'G', r.get('kernel'), r.get('avg_us'))" | tee -a gpurun_out/r05q_ab.txt
  done
done
