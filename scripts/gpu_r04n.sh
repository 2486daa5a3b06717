#!/bin/bash
# Round 4: the issue-cost probe with more instruction forms; the whole -m gpu suite + smoke after the scalar
# block-boundary count; C4 / C5 single-stream frames (k_resample per-kernel time against profiles/r04/merged_group_top_ab.txt).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 ./scripts/isa_rates.bin > gpurun_out/r04n_isa_rates.txt 2>&1 || { cat gpurun_out/r04n_isa_rates.txt; exit 1; }
cat gpurun_out/r04n_isa_rates.txt
bash scripts/gpu_suite.sh || exit 1
for c in C4 C5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 40 --warmup 5 --cpu-frames 0 --worst-frames 0 \
    --multi-sweep none --scale-ref-steps 0 --exact-steps 0 --single-points none > gpurun_out/r04n_$c.log 2>&1 || { tail -5 gpurun_out/r04n_$c.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04n_$c.log').read().strip().splitlines()[-1])
print('$c', round(d['ms_per_step']*1e3,1), 'us', round(d['value']/1e9,2), 'G', d['roofline']['per_kernel_avg_us'])"
done
