#!/bin/bash
# Round-2 confirmation from a rebuilt tree: the whole -m gpu suite, smoke, the default bench line and a C4
# bench line.  Every GPU step has its own time limit; steps are chained with && (stop at the first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
tag=${TAG:-r02_confirm}
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/${tag}_gpu_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/${tag}_bench_c2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config C4 --cpu-frames 0 --steps 50 --warmup 5 > gpurun_out/${tag}_bench_c4.log 2>&1
rc=$?
tail -3 gpurun_out/${tag}_gpu_tests.log
cat gpurun_out/${tag}_bench_c2.log gpurun_out/${tag}_bench_c4.log 2>/dev/null | cut -c1-600
exit $rc
