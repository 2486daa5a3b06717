#!/bin/bash
# Round 5 (aw): k_resample_final's winner-key maximum as two 32-bit DPP maxima (was 64-bit lane shuffles):
# the tests of the two-launch path, then C4 / C5 A/B
# against the previous build (records compared).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 170 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_frame_shapes.py tests/test_gpu_weigh_pk.py tests/test_gpu_resample_counts.py tests/test_gpu_defer.py \
  tests/test_gpu_packed_oracle.py tests/test_gpu_multi.py tests/test_gpu_resample_owners.py tests/test_gpu_parity.py \
  > gpurun_out/r05aw_tests.log 2>&1 || { tail -30 gpurun_out/r05aw_tests.log; exit 1; }
tail -3 gpurun_out/r05aw_tests.log
AB_CONFIGS="C4 C5" AB_LIBS="base=ab/libpfmpe_base.so new=" bash scripts/ab_libs.sh > gpurun_out/r05aw_ab.txt 2>&1 || { cat gpurun_out/r05aw_ab.txt; exit 1; }
cat gpurun_out/r05aw_ab.txt
