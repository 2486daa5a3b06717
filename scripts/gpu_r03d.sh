#!/bin/bash
# Round 3, fourth pass: the whole -m gpu suite + smoke, A/B against ab/libpfmpe_base.so on C4 / C5 / C3 and on
# batched C2 streams (16 / 32, one and two concurrent batches); records must be identical.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
bash scripts/gpu_suite.sh || exit 1
AB_CONFIGS="C4 C5 C3" bash scripts/ab_r03.sh > gpurun_out/ab_r03d.log 2>&1; rc=$?; cat gpurun_out/ab_r03d.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_multi_r03.sh > gpurun_out/ab_r03d_multi.log 2>&1; rc=$?; cat gpurun_out/ab_r03d_multi.log; exit $rc
