#!/bin/bash
# Round 5 (g): k_resample_owners with several blocks per wave: identity, then frame times at C4 / C5 for blocks per
# wave 1 / 2 / 4 / auto against the block-per-256 k_resample (no HIP events, two rounds), PMC at C4 (auto).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_resample_owners.py -x -q --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/r05g_tests.log 2>&1 || { tail -30 gpurun_out/r05g_tests.log; exit 1; }
tail -n 2 gpurun_out/r05g_tests.log
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
  for cfg in C4 C5; do
    for v in auto 1 2 4 blk; do
      case $v in auto) a="";; blk) a="--diag 32768";; *) a="--owners-bpw $v";; esac
      timeout -k 10 300 python -u bench.py --config $cfg $a --no-timing --steps 200 --warmup 20 $common > gpurun_out/r05g_${cfg}_$v.log 2>&1 || { tail -5 gpurun_out/r05g_${cfg}_$v.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('gpurun_out/r05g_${cfg}_$v.log').read().strip().splitlines()[-1])
print('$cfg $v no-timing', round(d['ms_per_step']*1e3,2), 'us', round(d['value']/1e9,3), 'G')" | tee -a gpurun_out/r05g_ab.txt
    done
  done
done
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d gpurun_out/r05g_pmc -o run -- python3 bench.py --config C4 --no-timing $common --steps 10 --warmup 2 > gpurun_out/r05g_pmc.log 2>&1 || { tail -5 gpurun_out/r05g_pmc.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/r05g_pmc > gpurun_out/r05g_pmc.txt 2>&1
grep -A9 "k_resample_owners" gpurun_out/r05g_pmc.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05g_tr -o run -- python3 bench.py --config C4 --no-timing $common --steps 50 --warmup 5 > gpurun_out/r05g_tr.log 2>&1 || { tail -5 gpurun_out/r05g_tr.log; exit 1; }
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/r05g_tr/run_kernel_stats.csv')):
    print('%-40s %5s %9.2f us' % (r['Name'].split('(')[0][-40:], r['Calls'], float(r['AverageNs']) / 1e3))
PY
