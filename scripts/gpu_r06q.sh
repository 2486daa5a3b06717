#!/bin/bash
# Round 6 (q): recovery after an abandoned finish (reset_handoffs): the two new tests, then the owners and batch suites
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_resample_owners.py::test_owners_abandoned_finish_leaves_no_state" \
  "tests/test_gpu_multi.py::test_multi_abandoned_finish_leaves_no_state" \
  tests/test_gpu_resample_owners.py tests/test_gpu_multi.py > gpurun_out/r06/tests_q.log 2>&1; r=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r06/tests_q.log | tail -40
exit $r
