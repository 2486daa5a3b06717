#!/bin/bash
# A/B of bench argument sets on the in-tree library, alternating (AB_SETS: ';'-separated argument sets)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
IFS=';' read -ra SETS <<< "${AB_SETS:---prune 1;--prune 0}"
for r in 1 2 3; do
  i=0
  for a in "${SETS[@]}"; do
    timeout -k 10 300 python bench.py --cpu-frames 0 --steps 400 --warmup 40 $a > gpurun_out/aba_$i.log 2>&1 || { tail gpurun_out/aba_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/aba_$i.log')); print('[$a]', round(d['ms_per_step']*1e3,2), 'us/frame', d['roofline']['per_kernel_avg_us'])"
    i=$((i+1))
  done
done
