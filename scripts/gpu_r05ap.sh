#!/bin/bash
# Round 5 (ak): group_math2's block argmax as integer reductions on fp32 keys (wave_argmax_f32key): the tests that
# check pairs against the oracle / across shapes, then the C2 A/B against the previous build and both builds' phase
# stamps (the winner candidate is on the C2 chain).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -q --timeout 170 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_frame_shapes.py tests/test_gpu_resident.py \
  tests/test_gpu_closed_loop.py tests/test_gpu_packed_oracle.py tests/test_gpu_resample_owners.py \
  tests/test_gpu_multi.py > gpurun_out/r05ap_tests.log 2>&1 || { tail -30 gpurun_out/r05ap_tests.log; exit 1; }
tail -3 gpurun_out/r05ap_tests.log
AB_CONFIGS="C2" AB_LIBS="base=ab/libpfmpe_base.so new=" bash scripts/ab_libs.sh > gpurun_out/r05ap_ab.txt 2>&1 || { cat gpurun_out/r05ap_ab.txt; exit 1; }
cat gpurun_out/r05ap_ab.txt
PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_base.so timeout -k 10 120 python -u scripts/diag_stamps.py 100000 > gpurun_out/r05ap_stamps_base.txt 2>&1 || exit 1
timeout -k 10 120 python -u scripts/diag_stamps.py 100000 > gpurun_out/r05ap_stamps_new.txt 2>&1 || exit 1
paste gpurun_out/r05ap_stamps_base.txt gpurun_out/r05ap_stamps_new.txt | cut -c1-140 | head -31
