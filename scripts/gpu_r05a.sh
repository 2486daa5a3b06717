#!/bin/bash
# Round 5 (a): k_resample_owners (one wave per 256-particle block) — identity against the block-per-256 k_resample,
# then an alternating A/B of the two (PFMPE_DIAG 32768 = DIAG_BLOCK_RESAMPLE) at C4 / C5 / C3, then the SALU /
# VALU counts of both at C4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_resample_owners.py tests/test_gpu_defer.py -x -v --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/r05a_tests.log 2>&1 || { tail -30 gpurun_out/r05a_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r05a_tests.log | tail -3
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0 --steps 100 --warmup 10"
for r in 1 2; do
  for cfg in C4 C5 C3; do
    for d in 0 32768; do
      timeout -k 10 300 python -u bench.py --config $cfg --diag $d $common > gpurun_out/r05a_${cfg}_$d.log 2>&1 || { tail -5 gpurun_out/r05a_${cfg}_$d.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('gpurun_out/r05a_${cfg}_$d.log').read().strip().splitlines()[-1])
print('$cfg diag $d', round(d['ms_per_step']*1e3,2), 'us', round(d['value']/1e9,3), 'G', d['roofline'].get('per_kernel_avg_us'))" | tee -a gpurun_out/r05a_ab.txt
    done
  done
done
for d in 0 32768; do
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d gpurun_out/r05a_pmc_$d -o run -- python3 bench.py --config C4 --diag $d --no-timing --cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0 --steps 10 --warmup 2 > gpurun_out/r05a_pmc_$d.log 2>&1 || { tail -5 gpurun_out/r05a_pmc_$d.log; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/r05a_pmc_0 > gpurun_out/r05a_pmc_0.txt 2>&1; python3 scripts/pmc_summary.py gpurun_out/r05a_pmc_32768 > gpurun_out/r05a_pmc_32768.txt 2>&1
grep -E "k_resample" gpurun_out/r05a_pmc_*.txt | head -20
exit 0
