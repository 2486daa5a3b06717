#!/bin/bash
# Round 3, fifth pass: the -m gpu suite + smoke; the batched path three times over (C2 streams S = 8 / 16 / 32 as one
# and two concurrent batches, then 8 C5 streams as two batches); A/B against ab/libpfmpe_base.so on C4 / C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
bash scripts/gpu_suite.sh || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --config C2 --steps 20 --warmup 5 --cpu-frames 0 --worst-frames 0 --scale-ref-steps 0 \
    --exact-steps 0 --multi-sweep 8,16,32 --multi-groups 1,2 --multi-steps 100 > gpurun_out/multi_stress_$r.log 2>&1 || { grep -a -v "^\s" gpurun_out/multi_stress_$r.log | tail -5; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/multi_stress_$r.log').read().strip().splitlines()[-1])
print('run $r', ' | '.join(f\"S{p['streams']}G{p['groups']} {p['ms_per_batch']*1e3:.1f}us {p['frac']}\" for p in d['multi_stream']['points']))"
done
timeout -k 10 300 python -u bench.py --config C5 --steps 20 --warmup 5 --cpu-frames 0 --worst-frames 0 --scale-ref-steps 0 \
  --exact-steps 0 --multi-sweep 8 --multi-groups 2 --multi-steps 50 > gpurun_out/multi_stress_c5.log 2>&1 || { grep -a -v "^\s" gpurun_out/multi_stress_c5.log | tail -5; exit 1; }
echo "C5 x 8 as two batches OK"
AB_CONFIGS="C4 C5" bash scripts/ab_r03.sh > gpurun_out/ab_r03e.log 2>&1; rc=$?; cat gpurun_out/ab_r03e.log; exit $rc
