#!/bin/bash
# quick GPU loop: parity tests, phase stamps (fused and two-launch), bench (each step time-limited;
# stop on the first failure)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
PFMPE_FUSED=1 timeout -k 10 300 python scripts/diag_stamps.py ${STAMP_N:-100000} > gpurun_out/stamps.log 2>&1 || { cat gpurun_out/stamps.log; exit 1; }
cat gpurun_out/stamps.log
PFMPE_FUSED=0 timeout -k 10 300 python scripts/diag_stamps.py ${STAMP_N:-100000 1000000} > gpurun_out/stamps2.log 2>&1 || { cat gpurun_out/stamps2.log; exit 1; }
cat gpurun_out/stamps2.log
timeout -k 10 300 python bench.py --cpu-frames 0 > gpurun_out/bench.log 2>&1 || { tail gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.log
