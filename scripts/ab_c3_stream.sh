#!/bin/bash
# C3 (12 markers, 200 heavy blobs, 1M): the one-block weighing pass (forced by PFMPE_DIAG 512; the default for > 8
# markers until round 3) against the streaming pass (the default now), alternating, two rounds; records compared.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
COMMON="--config C3 --steps 100 --warmup 10 --cpu-frames 0 --worst-frames 0 --multi-sweep none"
for r in 1 2; do
  for v in block stream; do
    d=""; [ $v = block ] && d="--diag 512"
    timeout -k 10 200 python -u bench.py $COMMON $d --dump-records gpurun_out/rec_c3_$v > gpurun_out/abc3_$v.log 2>&1 || { tail -3 gpurun_out/abc3_$v.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/abc3_$v.log').read().strip().splitlines()[-1]); print('C3 $v', round(d['ms_per_step']*1e3,2), 'us/frame', d['roofline']['per_kernel_avg_us'])"
  done
done
if cmp -s gpurun_out/rec_c3_block.0.json gpurun_out/rec_c3_stream.0.json; then echo "C3 records identical"; else echo "C3 RECORDS DIFFER"; fi
