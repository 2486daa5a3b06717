#!/bin/bash
# Round 6 (r): the owners finisher stages the frame constants and touches the blob table's lines before polling
# the arrivals (tree) against the previous build (ab/libpfmpe_base.so): owners tests, then C5 / C3 / C4 twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_resample_owners.py "tests/test_gpu_multi.py::test_multi_equals_single_streams" > gpurun_out/r06/tests_r.log 2>&1 || { tail -30 gpurun_out/r06/tests_r.log; exit 1; }
tail -n 1 gpurun_out/r06/tests_r.log
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
for cfg in C5 C3 C4; do
  for v in tree base; do
    if [ $v = tree ]; then unset PFMPE_LIB_OVERRIDE; else export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_$v.so; fi
    timeout -k 10 200 python -u bench.py --config $cfg --steps 300 --warmup 10 $common > gpurun_out/r06/ab_r_$v.log 2>&1 || { tail -5 gpurun_out/r06/ab_r_$v.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06/ab_r_$v.log').read().splitlines() if l.startswith('{')][-1])
r=d['roofline']; print('$cfg $v', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,2), 'G', r['per_kernel_avg_us'])" | tee -a gpurun_out/r06/ab_r.txt
  done
done
done
unset PFMPE_LIB_OVERRIDE
