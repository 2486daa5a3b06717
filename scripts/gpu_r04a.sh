#!/bin/bash
# Round 4, first GPU pass: the new parity tests (exact stratified counts at C2-C5 sizes, fp16 closed loops,
# 60-frame C2 closed loop), then the C4 / C5 single-stream benches as this round's starting point.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_resample_counts.py tests/test_gpu_closed_loop.py -x -v -s \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04a_tests.log 2>&1; r=$?
grep -E "PASS|FAIL|ERROR|frames within|C[2-5] \[|passed|failed" gpurun_out/r04a_tests.log | tail -30
[ $r -eq 0 ] || exit $r
for c in C4 C5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 100 --warmup 10 --cpu-frames 0 --worst-frames 0 --scale-ref-steps 0 \
    --exact-steps 0 --multi-sweep none > gpurun_out/r04a_bench_$c.log 2>&1 || { tail -5 gpurun_out/r04a_bench_$c.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04a_bench_$c.log').read().strip().splitlines()[-1])
print('$c', round(d['ms_per_step']*1e3,1), 'us/frame', round(d['value']/1e9,2), 'G/s', d['roofline'].get('per_kernel_avg_us'))"
done
