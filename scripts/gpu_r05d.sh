#!/bin/bash
# Round 5 (d): k_resample_owners with the direct owner writes: identity, then frame times of the occupancy floors
# 8 (in-tree) / 7 / 6 (ab/libpfmpe_w7.so, ab/libpfmpe_w6.so) at C4 / C5 without HIP events (two alternating rounds),
# one event-timed run each for the per-kernel averages, and the per-frame look at C5's heavy frames.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_resample_owners.py -x -q --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/r05d_tests.log 2>&1 || { tail -30 gpurun_out/r05d_tests.log; exit 1; }
tail -n 2 gpurun_out/r05d_tests.log
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
  for cfg in C4 C5; do
    for v in w8 w7 w6 blk; do
      d=0
      case $v in w8) unset PFMPE_LIB_OVERRIDE;; blk) unset PFMPE_LIB_OVERRIDE; d=32768;; *) export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_$v.so;; esac
      timeout -k 10 300 python -u bench.py --config $cfg --diag $d --no-timing --steps 200 --warmup 20 $common > gpurun_out/r05d_${cfg}_$v.log 2>&1 || { tail -5 gpurun_out/r05d_${cfg}_$v.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('gpurun_out/r05d_${cfg}_$v.log').read().strip().splitlines()[-1])
print('$cfg $v no-timing', round(d['ms_per_step']*1e3,2), 'us', round(d['value']/1e9,3), 'G')" | tee -a gpurun_out/r05d_ab.txt
    done
  done
done
unset PFMPE_LIB_OVERRIDE
for cfg in C4 C5; do
  for v in w8 w7 w6; do
    case $v in w8) unset PFMPE_LIB_OVERRIDE;; *) export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_$v.so;; esac
    timeout -k 10 300 python -u bench.py --config $cfg --steps 200 --warmup 20 --timing-period 10 $common > gpurun_out/r05d_ev_${cfg}_$v.log 2>&1 || { tail -5 gpurun_out/r05d_ev_${cfg}_$v.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r05d_ev_${cfg}_$v.log').read().strip().splitlines()[-1])
print('$cfg $v events', round(d['ms_per_step']*1e3,2), 'us', d['roofline'].get('per_kernel_avg_us'))" | tee -a gpurun_out/r05d_ab.txt
  done
done
unset PFMPE_LIB_OVERRIDE
timeout -k 10 250 python -u scripts/diag_owners.py C5 60 > gpurun_out/r05d_c5.txt 2>&1 || { tail -5 gpurun_out/r05d_c5.txt; exit 1; }
tail -n 14 gpurun_out/r05d_c5.txt
