#!/bin/bash
# Round 5 (e): k_resample_owners with light per-lane / heavy whole-wave owner writes: identity, frame-time A/B against
# the block-per-256 k_resample at C4 / C5 (no HIP events, two rounds), the C5 heavy frames, a PMC pass at C4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_resample_owners.py -x -q --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/r05f_tests.log 2>&1 || { tail -30 gpurun_out/r05f_tests.log; exit 1; }
tail -n 2 gpurun_out/r05f_tests.log
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
  for cfg in C4 C5; do
    for d in 0 32768; do
      timeout -k 10 300 python -u bench.py --config $cfg --diag $d --no-timing --steps 200 --warmup 20 $common > gpurun_out/r05f_${cfg}_$d.log 2>&1 || { tail -5 gpurun_out/r05f_${cfg}_$d.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('gpurun_out/r05f_${cfg}_$d.log').read().strip().splitlines()[-1])
print('$cfg diag $d no-timing', round(d['ms_per_step']*1e3,2), 'us', round(d['value']/1e9,3), 'G')" | tee -a gpurun_out/r05f_ab.txt
    done
  done
done
timeout -k 10 250 python -u scripts/diag_owners.py C5 60 > gpurun_out/r05f_c5.txt 2>&1 || { tail -5 gpurun_out/r05f_c5.txt; exit 1; }
tail -n 16 gpurun_out/r05f_c5.txt
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d gpurun_out/r05f_pmc -o run -- python3 bench.py --config C4 --no-timing $common --steps 10 --warmup 2 > gpurun_out/r05f_pmc.log 2>&1 || { tail -5 gpurun_out/r05f_pmc.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/r05f_pmc > gpurun_out/r05f_pmc.txt 2>&1
grep -A9 "k_resample_owners" gpurun_out/r05f_pmc.txt
