#!/bin/bash
# Round 6 (m): the whole -m gpu suite and smoke() (run again on the final tree)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/gpu_suite_m.log 2>&1; r=$?
tail -n 30 gpurun_out/r06/gpu_suite_m.log | grep -v "^$" | tail -12
[ $r -eq 0 ] || exit $r
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06/smoke_m.log 2>&1; r=$?
tail -5 gpurun_out/r06/smoke_m.log
exit $r
