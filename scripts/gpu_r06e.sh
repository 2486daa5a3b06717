#!/bin/bash
# Round 6 (e): k_weigh_pk12 (C3's packed 12-marker pass): bit identity + oracle tests, then C3 A/B:
# new (3 waves, phases of 4), ab/libpfmpe_pk12w4.so (4 waves, phases of 2), ab/libpfmpe_r05.so (k_weigh_stream)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_weigh_pk.py tests/test_gpu_packed_oracle.py "tests/test_gpu_frame_shapes.py::test_streaming_weighing_is_bit_identical" \
  tests/test_gpu_closed_loop.py > gpurun_out/r06/tests_e.log 2>&1 || { tail -40 gpurun_out/r06/tests_e.log; exit 1; }
tail -n 1 gpurun_out/r06/tests_e.log
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
  for v in new pk12w4 r05; do
    if [ $v = new ]; then unset PFMPE_LIB_OVERRIDE; else export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_$v.so; fi
    timeout -k 10 200 python -u bench.py --config C3 --steps 200 --warmup 10 $common > gpurun_out/r06/ab_e_$v.log 2>&1 || { tail -5 gpurun_out/r06/ab_e_$v.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06/ab_e_$v.log').read().splitlines() if l.startswith('{')][-1])
r=d['roofline']; print('C3 $v', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,2), 'G', r['per_kernel_avg_us'])" | tee -a gpurun_out/r06/ab_e.txt
  done
done
unset PFMPE_LIB_OVERRIDE
