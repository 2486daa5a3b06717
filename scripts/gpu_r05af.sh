#!/bin/bash
# Round 5 (af): how much of k_frame2's group arithmetic the min-side chains cost (diagnostic variant, not a product
# build): C2 A/B + the phase stamps of both builds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
AB_CONFIGS=C2 AB_LIBS="new= nomin=ab/libpfmpe_nomin.so" bash scripts/ab_libs.sh > gpurun_out/r05af_ab.txt 2>&1 || { cat gpurun_out/r05af_ab.txt; exit 1; }
cat gpurun_out/r05af_ab.txt
timeout -k 10 120 python -u scripts/diag_stamps.py 100000 > gpurun_out/r05af_stamps_new.txt 2>&1 || exit 1
PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_nomin.so timeout -k 10 120 python -u scripts/diag_stamps.py 100000 > gpurun_out/r05af_stamps_nomin.txt 2>&1 || exit 1
paste gpurun_out/r05af_stamps_new.txt gpurun_out/r05af_stamps_nomin.txt | cut -c1-140
