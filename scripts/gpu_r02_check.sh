#!/bin/bash
# Round-2 GPU check: the new shape / recovery / caller / two-rank tests first, then the whole -m gpu suite,
# smoke and a default bench line.  Every GPU step has its own time limit; steps are chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_frame_shapes.py tests/test_gpu_capi_caller.py tests/test_bench_dist.py > gpurun_out/r02_new_tests.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r02_gpu_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r02_bench_c2.log 2>&1
