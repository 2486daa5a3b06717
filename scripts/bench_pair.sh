#!/bin/bash
# bench: C loop vs Python loop, same workload (each its own time limit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --cpu-frames 0 > gpurun_out/bench_c.log 2>&1 || { tail gpurun_out/bench_c.log; exit 1; }
timeout -k 10 300 python bench.py --cpu-frames 0 --python-loop > gpurun_out/bench_py.log 2>&1 || { tail gpurun_out/bench_py.log; exit 1; }
timeout -k 10 300 python bench.py --cpu-frames 0 --no-timing > gpurun_out/bench_nt.log 2>&1 || { tail gpurun_out/bench_nt.log; exit 1; }
for f in c py nt; do python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_$f.log')); print('$f', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,3), 'G/s', d['roofline'] and d['roofline']['per_kernel_avg_us'])"; done
