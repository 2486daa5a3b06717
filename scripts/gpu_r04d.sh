#!/bin/bash
# Round 4, PMC passes of the batched path: 32 x C5 as two concurrent batches and 2 x C4 as one
# batch, each counter set in its own rocprofv3 run (scripts/pmc.sh), summaries to gpurun_out/pmc_r04_*.{txt,json}.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
common="--steps 5 --warmup 2 --worst-frames 0 --scale-ref-steps 0 --exact-steps 0 --single-points none --multi-steps 10"
bash scripts/pmc.sh r04_c5x32 --config C5 $common --multi-sweep 32 --multi-groups 2 > gpurun_out/pmc_r04_c5x32.txt 2>&1 \
  || { tail -20 gpurun_out/pmc_r04_c5x32.txt; exit 1; }
bash scripts/pmc.sh r04_c4x2 --config C4 $common --multi-sweep 2 --multi-groups 1 > gpurun_out/pmc_r04_c4x2.txt 2>&1 \
  || { tail -20 gpurun_out/pmc_r04_c4x2.txt; exit 1; }
bash scripts/pmc.sh r04_c4 --config C4 --steps 20 --warmup 3 --worst-frames 0 --multi-sweep none --single-points none \
  > gpurun_out/pmc_r04_c4.txt 2>&1 || { tail -20 gpurun_out/pmc_r04_c4.txt; exit 1; }
bash scripts/pmc.sh r04_c5 --config C5 --steps 20 --warmup 3 --worst-frames 0 --multi-sweep none --single-points none \
  > gpurun_out/pmc_r04_c5.txt 2>&1 || { tail -20 gpurun_out/pmc_r04_c5.txt; exit 1; }
grep -E "^k_|=> HBM|SQ_INSTS_VALU |SQ_WAVES " gpurun_out/pmc_r04_c5x32.txt gpurun_out/pmc_r04_c4x2.txt \
  gpurun_out/pmc_r04_c4.txt gpurun_out/pmc_r04_c5.txt
