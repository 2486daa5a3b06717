#!/bin/bash
# The PMC passes bench.py reads (profiles/pmc_<config>_n<N>.json: HBM traffic = 2 FETCH_SIZE + WRITE_SIZE, and the
# issue roofline's SQ_INSTS_VALU / SQ_INSTS_SALU), one config each, three counter passes per config (each its own
# rocprofv3 run, counters only, no trace domains; MI355X_MICROARCH.md HBM/rocprofv3 section).
#   bash scripts/pmc_lines.sh [C2 C3 C4 C5]   -> gpurun_out/pmc_<cfg>.json (copy to profiles/ to commit)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in ${@:-C2 C3 C4 C5}; do
  lc=$(echo $cfg | tr A-Z a-z)
  case $cfg in C2) st=40;; C5) st=20;; *) st=10;; esac
  args="--config $cfg --cpu-frames 0 --no-timing --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0 --steps $st --warmup 3"
  rm -rf gpurun_out/pmcl_$lc
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -k 10 180 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmcl_$lc/p$i -o run -- python3 bench.py $args > gpurun_out/pmcl_${lc}_p$i.log 2>&1 || { echo "pmc $cfg pass $i failed"; tail -5 gpurun_out/pmcl_${lc}_p$i.log; exit 1; }
  done
  python3 scripts/pmc_summary.py gpurun_out/pmcl_$lc --json gpurun_out/pmc_$lc.json > gpurun_out/pmcl_$lc.txt || exit 1
  echo "pmc $cfg done"
done
