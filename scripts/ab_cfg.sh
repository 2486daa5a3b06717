#!/bin/bash
# GPU tests, then A/B of the in-tree library against ab/libpfmpe_base.so over configs (alternating,
# each bench time-limited; stop on the first failure)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
for cfg in ${CONFIGS:-C4 C3 C2}; do
  st=50; [ $cfg = C2 ] && st=400
  for r in 1 2 3; do
    for v in base new; do
      if [ $v = base ]; then export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_base.so; else unset PFMPE_LIB_OVERRIDE; fi
      timeout -k 10 300 python bench.py --config $cfg --cpu-frames 0 --steps $st --warmup 5 ${AB_EXTRA} > gpurun_out/ab_$v.log 2>&1 || { tail gpurun_out/ab_$v.log; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.log')); print('$cfg $v', round(d['ms_per_step']*1e3,2), 'us/frame', d['roofline']['per_kernel_avg_us'])"
    done
  done
done
unset PFMPE_LIB_OVERRIDE
