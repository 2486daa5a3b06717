#!/bin/bash
# Round 4, after the fp32 packed-pass scratch fix: the batched points (32 x C5 as two batches, 2 x C4 as one) and
# the C5 / 32 x C5 PMC passes again.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --config C5 --steps 20 --warmup 5 --cpu-frames 0 --worst-frames 0 \
    --multi-sweep 8,32 --multi-groups 2 --multi-steps 30 > gpurun_out/r04h_multi_C5_$rep.log 2>&1 || { tail -5 gpurun_out/r04h_multi_C5_$rep.log; exit 1; }
  timeout -k 10 300 python -u bench.py --config C4 --steps 20 --warmup 5 --cpu-frames 0 --worst-frames 0 \
    --multi-sweep 2 --multi-groups 1 --multi-steps 30 > gpurun_out/r04h_multi_C4_$rep.log 2>&1 || { tail -5 gpurun_out/r04h_multi_C4_$rep.log; exit 1; }
  for c in C5 C4; do python3 -c "
import json; d=json.loads(open('gpurun_out/r04h_multi_${c}_$rep.log').read().strip().splitlines()[-1])
print('$c single', round(d['ms_per_step']*1e3,1), 'us', round(d['value']/1e9,2), 'G/s |',
      [(p['streams'], p['groups'], round(p['updates_per_s']/1e9,2), p['frac'], round(p['ms_per_batch']*1e3,1)) for p in d['multi_stream']['points']])"; done
done
common="--steps 5 --warmup 2 --worst-frames 0 --scale-ref-steps 0 --exact-steps 0 --single-points none --multi-steps 10"
bash scripts/pmc.sh r04h_c5x32 --config C5 $common --multi-sweep 32 --multi-groups 2 > gpurun_out/pmc_r04h_c5x32.txt 2>&1 \
  || { tail -20 gpurun_out/pmc_r04h_c5x32.txt; exit 1; }
bash scripts/pmc.sh r04h_c5 --config C5 --steps 20 --warmup 3 --worst-frames 0 --multi-sweep none --single-points none \
  > gpurun_out/pmc_r04h_c5.txt 2>&1 || { tail -20 gpurun_out/pmc_r04h_c5.txt; exit 1; }
grep -A40 "k_weigh_pk" gpurun_out/pmc_r04h_c5.txt | grep -E "^k_|FETCH|WRITE|HBM" | head -8
