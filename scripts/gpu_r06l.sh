#!/bin/bash
# Round 6 (l): the packed passes' fused group / top hand-off (PkTail): identity tests, then C5 / C4 / C3 against the
# previous commit's library (ab/libpfmpe_head.so) and the round-start one
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_weigh_pk.py tests/test_gpu_packed_oracle.py "tests/test_gpu_frame_shapes.py::test_streaming_weighing_is_bit_identical" \
  tests/test_gpu_resample_counts.py > gpurun_out/r06/tests_l.log 2>&1 || { tail -40 gpurun_out/r06/tests_l.log; exit 1; }
tail -n 1 gpurun_out/r06/tests_l.log
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
for cfg in C5 C4 C3; do
  for v in new head r05; do
    if [ $v = new ]; then unset PFMPE_LIB_OVERRIDE; else export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_$v.so; fi
    timeout -k 10 200 python -u bench.py --config $cfg --steps 200 --warmup 10 $common > gpurun_out/r06/ab_l_$v.log 2>&1 || { tail -5 gpurun_out/r06/ab_l_$v.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06/ab_l_$v.log').read().splitlines() if l.startswith('{')][-1])
r=d['roofline']; print('$cfg $v', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,2), 'G', r['per_kernel_avg_us'])" | tee -a gpurun_out/r06/ab_l.txt
  done
done
done
unset PFMPE_LIB_OVERRIDE
