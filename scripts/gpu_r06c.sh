#!/bin/bash
# Round 6 (c): sharded arrivals in the fused owners finish: owners / multi / parity tests, then C3/C4/C5 points
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_resample_owners.py tests/test_gpu_packed_oracle.py tests/test_gpu_defer.py tests/test_gpu_resample_counts.py > gpurun_out/r06/tests_c.log 2>&1 || { tail -30 gpurun_out/r06/tests_c.log; exit 1; }
tail -n 2 gpurun_out/r06/tests_c.log
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for cfg in C5 C4 C3; do
  timeout -k 10 200 python -u bench.py --config $cfg --steps 100 --warmup 10 $common > gpurun_out/r06/pt_c_$cfg.log 2>&1 || { tail -5 gpurun_out/r06/pt_c_$cfg.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06/pt_c_$cfg.log').read().splitlines() if l.startswith('{')][-1])
r=d['roofline']; print('$cfg', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,2), 'G', r['per_kernel_avg_us'])"
done
