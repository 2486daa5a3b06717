#!/bin/bash
# GPU tests, then short benches of C2/C3/C4 (each step time-limited; stop on the first failure)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
for r in 1 2; do
for cfg in ${CONFIGS:-C2 C3 C4}; do
  st=50; [ $cfg = C2 ] && st=400
  timeout -k 10 300 python bench.py --config $cfg --cpu-frames 0 --steps $st --warmup 5 $BENCH_EXTRA > gpurun_out/bc_$cfg.log 2>&1 || { tail gpurun_out/bc_$cfg.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bc_$cfg.log')); print('$cfg', round(d['ms_per_step']*1e3,2), 'us/frame', d['roofline']['per_kernel_avg_us'])"
done
done
