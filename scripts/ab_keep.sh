#!/bin/bash
# A/B of PFMPE_OPT_KEEP_PROPAGATED (two-launch path: stored vs regenerated propagated set) at C4 and C3,
# after the GPU tests that cover it.  Each step time-limited; stop on the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for cfg in ${AB_CONFIGS:-C4 C3}; do
  for k in 1 0 1 0; do
    timeout -k 10 300 python bench.py --config $cfg --cpu-frames 0 --steps 50 --warmup 5 --keep-prop $k > gpurun_out/abk_${cfg}_$k.log 2>&1 || { tail gpurun_out/abk_${cfg}_$k.log; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/abk_${cfg}_$k.log')); print('$cfg keep=$k', round(d['ms_per_step']*1e3,2), 'us/frame', d['roofline']['per_kernel_avg_us'])"
  done
done
