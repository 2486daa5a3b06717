#!/bin/bash
# Round 6 (v): k_group + k_top_wide as one launch (k_group_top_wide, PFMPE_DIAG 262144): identity, then C4 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_weigh_pk.py::test_merged_wide_handoff_is_bit_identical" > gpurun_out/r06/tests_v.log 2>&1 || { grep -E "PASSED|FAILED|Error|assert" gpurun_out/r06/tests_v.log | tail -20; exit 1; }
grep -E "PASSED|passed" gpurun_out/r06/tests_v.log | tail -3
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2 3; do
  for d in 262144 0; do
    timeout -k 10 200 python -u bench.py --config C4 --steps 200 --warmup 10 --diag $d $common > gpurun_out/r06/ab_v_$d.log 2>&1 || { tail -5 gpurun_out/r06/ab_v_$d.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06/ab_v_$d.log').read().splitlines() if l.startswith('{')][-1])
r=d['roofline']; print('C4 diag $d', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,2), 'G', r['per_kernel_avg_us'])" | tee -a gpurun_out/r06/ab_v.txt
  done
done
