#!/bin/bash
# The streaming-vs-one-block identity case that failed (fp16, 1.2M, 12 markers, 200 heavy blobs) under three
# libraries: the in-tree build, ab/libpfmpe_varA.so, ab/libpfmpe_base.so; each run under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
T='tests/test_gpu_frame_shapes.py::test_streaming_weighing_is_bit_identical'
for v in new varA base; do
  if [ $v = new ]; then unset PFMPE_LIB_OVERRIDE; else export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_$v.so; fi
  timeout -k 10 300 python -u -m pytest "$T" -x -q --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/bisect_$v.log 2>&1
  rc=$?; echo "$v rc=$rc: $(tail -1 gpurun_out/bisect_$v.log)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
