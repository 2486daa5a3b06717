#!/bin/bash
# Round 4: A/B of the instruction cuts (base = ad3a3cc, before them; w7 = current with the kept-set k_resample floor
# at 7 waves per SIMD, no SGPR spills; new = in-tree, floor 8) on C4 / C5 / C2, records compared.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
AB_LIBS="base=ab/libpfmpe_base.so w7=ab/libpfmpe_w7.so new=" AB_CONFIGS="C4 C5 C2" bash scripts/ab_libs.sh 2>&1 | tee gpurun_out/r04p_ab.txt
