#!/bin/bash
# Round 4: the whole -m gpu suite + smoke after the k_resample / k_weigh_pk instruction cuts (scalar block-boundary
# count, band division behind a wave-uniform test, div_by_S, fixed-point wave scans); then C4 / C5 single-stream
# frames and the 32 x C5 / 2 x C4 batches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_suite.sh || exit 1
for c in C4 C5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 40 --warmup 5 --cpu-frames 0 --worst-frames 0 \
    --multi-sweep $([ $c = C4 ] && echo 2 || echo 32) --multi-groups $([ $c = C4 ] && echo 1 || echo 2) --multi-steps 20 \
    --scale-ref-steps 0 --exact-steps 0 --single-points none > gpurun_out/r04o_$c.log 2>&1 || { tail -5 gpurun_out/r04o_$c.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04o_$c.log').read().strip().splitlines()[-1])
print('$c', round(d['ms_per_step']*1e3,1), 'us', round(d['value']/1e9,2), 'G', d['roofline']['per_kernel_avg_us'], '|',
      [(p['streams'], p['groups'], round(p['updates_per_s']/1e9,2), p['frac'], round(p['ms_per_batch']*1e3,1)) for p in d['multi_stream']['points']])"
done
