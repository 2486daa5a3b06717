#!/bin/bash
# Round 5 (x): batches: block map kept, lazy fence, one-stream-at-a-time packed weighing (seq) vs side by side
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_resample_owners.py::test_owners_batch_equals_block_resample -x -q --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/r05x_tests.log 2>&1 || { tail -30 gpurun_out/r05x_tests.log; exit 1; }
tail -n 1 gpurun_out/r05x_tests.log
for r in 1 2; do
  for d in 0 131072; do
    timeout -k 10 300 python -u scripts/diag_multi_host.py --diag $d > gpurun_out/r05x_$d.txt 2>&1 || { cat gpurun_out/r05x_$d.txt; exit 1; }
    echo "diag=$d $(head -1 gpurun_out/r05x_$d.txt)" | tee -a gpurun_out/r05x_ab.txt
  done
done
common="--cpu-frames 0 --worst-frames 0 --single-points C4 --single-steps 100 --scale-ref-steps 0 --exact-steps 0 --multi-sweep none"
timeout -k 10 600 python -u bench.py --steps 200 --warmup 20 $common > gpurun_out/r05x_bench.log 2>&1 || { tail -5 gpurun_out/r05x_bench.log; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/r05x_bench.log').read().strip().splitlines()[-1])
print('C2', round(d['ms_per_step']*1e3,2), 'us;', 'C4 single', round(d['single_stream']['C4']['value']/1e9,2), 'G')
PY
