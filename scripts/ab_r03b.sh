#!/bin/bash
# Round 3 (second pass): 4-way A/B on C4 / C5 (base = start of the pass, new, new without the single-barrier
# streaming loop, new without the packed fp16 stores), then one PMC pass of the instruction counts at C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
AB_LIBS="base=ab/libpfmpe_base.so new= bar=ab/libpfmpe_bar.so store=ab/libpfmpe_store.so" AB_CONFIGS="C4 C5" \
  bash scripts/ab_libs.sh || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVE_CYCLES \
  --output-format csv -d gpurun_out/pmcv_c4 -o run -- python3 bench.py --config C4 --cpu-frames 0 --no-timing --worst-frames 0 \
  --multi-sweep none --scale-ref-steps 0 --exact-steps 0 --steps 20 --warmup 3 > gpurun_out/pmcv_c4.log 2>&1 || { tail gpurun_out/pmcv_c4.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmcv_c4 > gpurun_out/pmcv_c4.txt 2>&1; grep -A9 -E "^k_(resample|weigh_stream)$" gpurun_out/pmcv_c4.txt
