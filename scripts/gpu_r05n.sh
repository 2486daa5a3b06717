#!/bin/bash
# Round 5 (n): resident server idle-poll sleep A/B (16 in-tree, 4, 64) at C2: device duration, phases, bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
  for v in s16 s4 s64; do
    case $v in s16) unset PFMPE_LIB_OVERRIDE;; s4) export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_sleep4.so;; s64) export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_sleep64.so;; esac
    timeout -k 10 200 python -u scripts/diag_resident.py > gpurun_out/r05n_${v}_$r.txt 2>&1 || { cat gpurun_out/r05n_${v}_$r.txt; exit 1; }
    for res in 1 0; do
      timeout -k 10 200 python -u bench.py --resident $res --steps 2000 --warmup 50 $common > gpurun_out/r05n_b_${v}_${res}.log 2>&1 || { tail -5 gpurun_out/r05n_b_${v}_${res}.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('gpurun_out/r05n_b_${v}_${res}.log').read().strip().splitlines()[-1])
r=d.get('roofline') or {}
print('$v resident=$res', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,3), 'G', r.get('kernel'), r.get('avg_us'))" | tee -a gpurun_out/r05n_ab.txt
    done
  done
done
unset PFMPE_LIB_OVERRIDE
grep -H "resident=" gpurun_out/r05n_s*_1.txt gpurun_out/r05n_s*_2.txt
cat gpurun_out/r05n_s16_2.txt
