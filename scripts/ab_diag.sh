#!/bin/bash
# A/B of diagnostic switches (bench --diag) on the in-tree library, alternating; each run time-limited
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for r in 1 2 3; do
  for d in ${AB_DIAGS:-0 64 128}; do
    timeout -k 10 300 python bench.py --cpu-frames 0 --steps 400 --warmup 40 --diag $d > gpurun_out/abd_$d.log 2>&1 || { tail gpurun_out/abd_$d.log; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/abd_$d.log')); print('diag $d', round(d['ms_per_step']*1e3,2), 'us/frame', d['roofline']['per_kernel_avg_us'])"
  done
done
