#!/bin/bash
# Round 6 (f): PMC passes of C3's weighing pass: k_weigh_pk12 (new) against k_weigh_stream (ab/libpfmpe_r05.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
args="--config C3 --cpu-frames 0 --no-timing --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0 --steps 10 --warmup 3"
for v in new r05; do
  if [ $v = new ]; then unset PFMPE_LIB_OVERRIDE; else export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_$v.so; fi
  rm -rf gpurun_out/r06/pmc3_$v; i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU_TRANS_F32 SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/r06/pmc3_$v/p$i -o run -- python3 bench.py $args > gpurun_out/r06/pmc3_${v}_p$i.log 2>&1 || { echo "pmc $v pass $i failed"; tail -5 gpurun_out/r06/pmc3_${v}_p$i.log; exit 1; }
  done
  python3 scripts/pmc_summary.py gpurun_out/r06/pmc3_$v > gpurun_out/r06/pmc3_$v.txt
  grep -A20 "k_weigh" gpurun_out/r06/pmc3_$v.txt | head -22
done
unset PFMPE_LIB_OVERRIDE
