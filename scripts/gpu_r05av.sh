#!/bin/bash
# Round 5 (av, experiment): does the host's record polling slow the resident server's back-to-back frames?  C2 2,000
# frames: launched, resident, resident with the host leaving the record alone for 15 us after each doorbell
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0 --no-timing"
for r in 1 2; do
  for v in launched resident backoff; do
    extra=""; unset PFMPE_LIB_OVERRIDE
    [ $v != launched ] && extra="--resident 1"
    [ $v = backoff ] && export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_backoff.so
    timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 $common $extra > gpurun_out/r05av_$v.log 2>&1 || { tail -5 gpurun_out/r05av_$v.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r05av_$v.log').read().strip().splitlines()[-1])
print('$v', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,3), 'G', d['config'].get('frame_shape'))" | tee -a gpurun_out/r05av_ab.txt
  done
done
