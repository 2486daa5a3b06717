#!/bin/bash
# Round 5 (au): the resident frame server against launched frames on the final tree (phases + C2 2,000-frame lines)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/diag_resident.py > gpurun_out/r05au_diag.txt 2>&1 || { cat gpurun_out/r05au_diag.txt; exit 1; }
head -3 gpurun_out/r05au_diag.txt; grep -A1 "resident=0" gpurun_out/r05au_diag.txt
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
  for v in launched resident; do
    extra=""; [ $v = resident ] && extra="--resident 1"
    timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 $common $extra > gpurun_out/r05au_$v.log 2>&1 || { tail -5 gpurun_out/r05au_$v.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r05au_$v.log').read().strip().splitlines()[-1])
print('$v', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,3), 'G', d['config'].get('frame_shape'))" | tee -a gpurun_out/r05au_ab.txt
  done
done
