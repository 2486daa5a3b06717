#!/bin/bash
# Round 6 (h): the combined A/B grid walk of k_weigh_pk12, and a 4x finer blob grid (ab/libpfmpe_cells8k.so:
# PFMPE_GRID_MAX_CELLS=8192): bit identity for both, then C3 / C2 / C5 / C4 against the round-start library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_weigh_pk.py > gpurun_out/r06/tests_h.log 2>&1 || { tail -30 gpurun_out/r06/tests_h.log; exit 1; }
tail -n 1 gpurun_out/r06/tests_h.log
PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_cells8k.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_weigh_pk.py tests/test_gpu_grid_far.py tests/test_gpu_grid_lists.py > gpurun_out/r06/tests_h8k.log 2>&1 || { tail -30 gpurun_out/r06/tests_h8k.log; exit 1; }
tail -n 1 gpurun_out/r06/tests_h8k.log
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
for cfg in C3 C2 C5 C4; do
  for v in new cells8k r05; do
    if [ $v = new ]; then unset PFMPE_LIB_OVERRIDE; else export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_$v.so; fi
    st=200; [ $cfg = C2 ] && st=1000
    timeout -k 10 200 python -u bench.py --config $cfg --steps $st --warmup 10 $common > gpurun_out/r06/ab_h_$v.log 2>&1 || { tail -5 gpurun_out/r06/ab_h_$v.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06/ab_h_$v.log').read().splitlines() if l.startswith('{')][-1])
r=d['roofline']; print('$cfg $v', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,2), 'G', r['per_kernel_avg_us'])" | tee -a gpurun_out/r06/ab_h.txt
  done
done
done
unset PFMPE_LIB_OVERRIDE
