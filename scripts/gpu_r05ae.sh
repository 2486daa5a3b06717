#!/bin/bash
# Round 5 (ae): k_weigh_pk with the loop conditions pinned per task (fewer SGPR spills): tests + C4/C5 A/B + PMC
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_weigh_pk.py tests/test_gpu_multi.py -x -q --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/r05ae_tests.log 2>&1 || { tail -30 gpurun_out/r05ae_tests.log; exit 1; }
tail -n 1 gpurun_out/r05ae_tests.log
AB_LIBS="new= base=ab/libpfmpe_base.so" AB_CONFIGS="C4 C5" timeout -k 10 800 bash scripts/ab_libs.sh > gpurun_out/r05ae_ab.txt 2>&1 || { tail -20 gpurun_out/r05ae_ab.txt; exit 1; }
grep -E "C4|C5" gpurun_out/r05ae_ab.txt
