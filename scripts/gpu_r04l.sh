#!/bin/bash
# Round 4: phase stamps of the two-launch frame at C4 (k_resample and k_resample_final timelines).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PFMPE_CFG=C4 PFMPE_FUSED=0 timeout -k 10 400 python -u scripts/diag_stamps.py 10000000 > gpurun_out/r04l_stamps_c4.log 2>&1 \
  || { tail -5 gpurun_out/r04l_stamps_c4.log; exit 1; }
cat gpurun_out/r04l_stamps_c4.log
PFMPE_CFG=C5 PFMPE_FUSED=0 timeout -k 10 400 python -u scripts/diag_stamps.py 1000000 > gpurun_out/r04l_stamps_c5.log 2>&1 \
  || { tail -5 gpurun_out/r04l_stamps_c5.log; exit 1; }
cat gpurun_out/r04l_stamps_c5.log
