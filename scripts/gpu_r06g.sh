#!/bin/bash
# Round 6 (g): k_weigh_pk without SGPR spills (packed-min dup test) + k_weigh_pk12: tests, A/B against the round-start
# library at C5 / C4 / C3, then PMC passes of C3 (new and round-start)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_weigh_pk.py tests/test_gpu_packed_oracle.py tests/test_gpu_multi.py > gpurun_out/r06/tests_g.log 2>&1 || { tail -40 gpurun_out/r06/tests_g.log; exit 1; }
tail -n 1 gpurun_out/r06/tests_g.log
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
for cfg in C5 C4 C3; do
  for v in new r05; do
    if [ $v = new ]; then unset PFMPE_LIB_OVERRIDE; else export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_$v.so; fi
    timeout -k 10 200 python -u bench.py --config $cfg --steps 200 --warmup 10 $common > gpurun_out/r06/ab_g_$v.log 2>&1 || { tail -5 gpurun_out/r06/ab_g_$v.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06/ab_g_$v.log').read().splitlines() if l.startswith('{')][-1])
r=d['roofline']; print('$cfg $v', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,2), 'G', r['per_kernel_avg_us'])" | tee -a gpurun_out/r06/ab_g.txt
  done
done
done
unset PFMPE_LIB_OVERRIDE
timeout -k 10 500 bash scripts/gpu_r06f.sh
