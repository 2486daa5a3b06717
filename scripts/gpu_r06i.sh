#!/bin/bash
# Round 6 (i): adaptive grid budget (fine grid from 128 blobs): the whole -m gpu suite, then C3 / C5 / C2 against the
# round-start library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/gpu_suite_i.log 2>&1; r=$?
tail -n 3 gpurun_out/r06/gpu_suite_i.log
[ $r -eq 0 ] || { grep -B5 -A30 "FAILURES" gpurun_out/r06/gpu_suite_i.log | head -60; exit $r; }
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
for cfg in C3 C5; do
  for v in new r05; do
    if [ $v = new ]; then unset PFMPE_LIB_OVERRIDE; else export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_$v.so; fi
    timeout -k 10 200 python -u bench.py --config $cfg --steps 200 --warmup 10 $common > gpurun_out/r06/ab_i_$v.log 2>&1 || { tail -5 gpurun_out/r06/ab_i_$v.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06/ab_i_$v.log').read().splitlines() if l.startswith('{')][-1])
r=d['roofline']; print('$cfg $v', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,2), 'G', r['per_kernel_avg_us'])" | tee -a gpurun_out/r06/ab_i.txt
  done
done
done
unset PFMPE_LIB_OVERRIDE
