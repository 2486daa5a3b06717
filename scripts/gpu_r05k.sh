#!/bin/bash
# Round 5 (k): the resident frame server (tests + C2 A/B), then (i)'s owners / batch / packed-oracle checks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05k_resident.log 2>&1 || { tail -40 gpurun_out/r05k_resident.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r05k_resident.log
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
  for v in res launch; do
    case $v in res) a="--resident 1";; launch) a="--resident 0";; esac
    timeout -k 10 200 python -u bench.py $a --steps 2000 --warmup 50 $common > gpurun_out/r05k_c2_$v.log 2>&1 || { tail -5 gpurun_out/r05k_c2_$v.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r05k_c2_$v.log').read().strip().splitlines()[-1])
r=d.get('roofline') or {}
print('C2 $v', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,3), 'G', r.get('kernel'), r.get('avg_us'))" | tee -a gpurun_out/r05k_ab.txt
  done
done
true
