#!/bin/bash
# Round 5 (m): resident server phases, write-through (in-tree) vs plain stores + release (ab/libpfmpe_srvplain.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 200 python -u scripts/diag_resident.py > gpurun_out/r05m_wt_$r.txt 2>&1 || { cat gpurun_out/r05m_wt_$r.txt; exit 1; }
  PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_srvplain.so timeout -k 10 200 python -u scripts/diag_resident.py > gpurun_out/r05m_plain_$r.txt 2>&1 || { cat gpurun_out/r05m_plain_$r.txt; exit 1; }
done
for f in gpurun_out/r05m_*_1.txt gpurun_out/r05m_*_2.txt; do echo "== $f"; cat $f; done
