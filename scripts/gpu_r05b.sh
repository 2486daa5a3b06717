#!/bin/bash
# Round 5 (b): kernel trace of k_resample_owners vs k_resample (C4, C5), and frame times without HIP events.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
  for cfg in C4 C5; do
    for d in 0 32768; do
      timeout -k 10 300 python -u bench.py --config $cfg --diag $d --no-timing --steps 200 --warmup 20 $common > gpurun_out/r05b_${cfg}_$d.log 2>&1 || { tail -5 gpurun_out/r05b_${cfg}_$d.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('gpurun_out/r05b_${cfg}_$d.log').read().strip().splitlines()[-1])
print('$cfg diag $d no-timing', round(d['ms_per_step']*1e3,2), 'us', round(d['value']/1e9,3), 'G')" | tee -a gpurun_out/r05b_ab.txt
    done
  done
done
for cfg in C4 C5; do
  for d in 0 32768; do
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05b_tr_${cfg}_$d -o run -- python3 bench.py --config $cfg --diag $d --no-timing --steps 50 --warmup 5 $common > gpurun_out/r05b_tr_${cfg}_$d.log 2>&1 || { tail -5 gpurun_out/r05b_tr_${cfg}_$d.log; exit 1; }
    f=$(ls gpurun_out/r05b_tr_${cfg}_$d/*kernel_stats.csv | head -1); echo "== $cfg $d"; cut -d, -f1-8 $f | head -12
  done
done
exit 0
