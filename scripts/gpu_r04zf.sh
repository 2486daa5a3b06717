#!/bin/bash
# Round 4 close: the whole -m gpu suite + smoke and the driver's default bench command on the final tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_suite.sh || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r04zf_bench.log 2>&1 || { tail -5 gpurun_out/r04zf_bench.log; exit 1; }
tail -c 600 gpurun_out/r04zf_bench.log
