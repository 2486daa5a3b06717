#!/bin/bash
# Round 3, third pass: the whole -m gpu suite + smoke, the copy roofline micro-benchmark, A/B against the pass's
# base library on C4 / C5 / C2 (records must be identical), each step under its own limit; stop at a failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
bash scripts/gpu_suite.sh || exit 1
timeout -k 10 120 ./scripts/micro/copy_roof > gpurun_out/copy_roof.log 2>&1 || { cat gpurun_out/copy_roof.log; exit 1; }
cat gpurun_out/copy_roof.log
AB_CONFIGS="${AB_CONFIGS:-C4 C5 C2}" bash scripts/ab_r03.sh > gpurun_out/ab_r03c.log 2>&1; rc=$?; cat gpurun_out/ab_r03c.log; exit $rc
