#!/bin/bash
# Round 5 (i): the owners kernel with buffer/saddr I/O (A/B against k_resample at C4 / C5), the packed path against
# the oracle at full size, and the closed loops (with their margins, -s) incl. the new two-launch packed loops.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_resample_owners.py tests/test_gpu_multi.py tests/test_gpu_defer.py -x -q --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/r05i_tests.log 2>&1 || { tail -30 gpurun_out/r05i_tests.log; exit 1; }
tail -n 2 gpurun_out/r05i_tests.log
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
  for cfg in C4 C5; do
    for v in new blk; do
      case $v in new) a="";; blk) a="--diag 32768";; esac
      timeout -k 10 300 python -u bench.py --config $cfg $a --no-timing --steps 200 --warmup 20 $common > gpurun_out/r05i_${cfg}_$v.log 2>&1 || { tail -5 gpurun_out/r05i_${cfg}_$v.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('gpurun_out/r05i_${cfg}_$v.log').read().strip().splitlines()[-1])
print('$cfg $v no-timing', round(d['ms_per_step']*1e3,2), 'us', round(d['value']/1e9,3), 'G')" | tee -a gpurun_out/r05i_ab.txt
    done
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_packed_oracle.py tests/test_gpu_closed_loop.py -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05i_parity.log 2>&1 || { tail -30 gpurun_out/r05i_parity.log; exit 1; }
grep -E "PASS|FAIL|frames within|oracle|kept iteration" gpurun_out/r05i_parity.log
