#!/bin/bash
# Round-3 measurement pass: the default bench line (C2 + cpu_baseline + worst case + multi-stream sweep),
# C3 / C4 / C5 lines, rocprofv3 kernel stats of C2, C4, C5 and a 16-stream C2 batch, the C4, C5 and 16-stream PMC
# passes, and the initialisation bench.  Every GPU step has its own time limit; a failure stops the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
t=${TAG:-r03}
run() {  # run <name> <limit-s> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$lim" "$@" > "gpurun_out/${t}_$name.log" 2>&1
  local rc=$?
  tail -c 300 "gpurun_out/${t}_$name.log"; echo
  if [ $rc -ne 0 ]; then echo "STOP after $name rc=$rc"; exit $rc; fi
}
pmc() {  # pmc <name> <bench args> -- counters per pass as separate runs
  local name=$1 args=$2; local i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVE_CYCLES" \
             "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    run pmc_${name}_p$i 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/${t}_pmc_$name/p$i -o run -- python3 bench.py --cpu-frames 0 --no-timing --worst-frames 0 $args
  done
  python3 scripts/pmc_summary.py gpurun_out/${t}_pmc_$name --json gpurun_out/${t}_pmc_$name.json > gpurun_out/${t}_pmc_$name.txt 2>&1
}
if [ "${PHASE:-A}" = A ]; then
run bench_c2 400 python -u bench.py
run bench_c2_driver 400 python -u bench.py --steps 20 --warmup 5 --cpu-frames 0  # the driver's flags
run bench_c3 200 python -u bench.py --config C3 --cpu-frames 0 --steps 50 --warmup 5 --multi-sweep 1,4
run bench_c4 200 python -u bench.py --config C4 --cpu-frames 0 --steps 50 --warmup 5
run bench_c5 200 python -u bench.py --config C5 --cpu-frames 0 --steps 100 --warmup 10 --multi-sweep 1,2,4,8
run prof_c2 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${t}_prof_c2 -o run --output-format csv -- python3 bench.py --cpu-frames 0 --no-timing --worst-frames 0
run prof_c4 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${t}_prof_c4 -o run --output-format csv -- python3 bench.py --config C4 --cpu-frames 0 --no-timing --worst-frames 0 --steps 30 --warmup 5
run prof_c5 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${t}_prof_c5 -o run --output-format csv -- python3 bench.py --config C5 --cpu-frames 0 --no-timing --worst-frames 0 --steps 50 --warmup 5
run prof_multi16 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${t}_prof_multi16 -o run --output-format csv -- python3 bench.py --cpu-frames 0 --no-timing --worst-frames 0 --steps 10 --warmup 2 --multi-sweep 16 --multi-steps 100
for p in c2 c4 c5 multi16; do python3 scripts/trace_summary.py gpurun_out/${t}_prof_$p 12 > gpurun_out/${t}_prof_${p}_summary.txt 2>&1; done
fi
if [ "${PHASE:-A}" = B ]; then
pmc c2 "--steps 50 --warmup 5 --multi-sweep none --exact-steps 0 --scale-ref-steps 0"
pmc c4 "--config C4 --steps 20 --warmup 3 --multi-sweep none"
pmc c5 "--config C5 --steps 20 --warmup 3 --multi-sweep none"
run init 200 python -u scripts/bench_init.py
echo "== done $(date +%T)"
fi
