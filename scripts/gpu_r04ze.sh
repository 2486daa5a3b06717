#!/bin/bash
# Round 4: the long-cell-list test of the phased one-launch minima (tests/test_gpu_grid_lists.py) with the grid tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_grid_lists.py tests/test_gpu_grid_far.py -m gpu -x -v --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/r04ze.log 2>&1; r=$?
tail -n 8 gpurun_out/r04ze.log
exit $r
