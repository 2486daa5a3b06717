#!/bin/bash
# Round 6 (u): the packed passes at tiny N (new identity cases)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_weigh_pk.py::test_pk_passes_small_n" > gpurun_out/r06/tests_u.log 2>&1; r=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/r06/tests_u.log | tail -20
exit $r
