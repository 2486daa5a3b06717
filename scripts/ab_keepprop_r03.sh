#!/bin/bash
# Keep-prop (PFMPE_OPT_KEEP_PROPAGATED) on / off per workload, alternating, two rounds: one-stream C5 / C4 / C3
# and the batched C2 x 32 (two batches) and C5 x 8 (two batches) points.  VERDICT r02 item 5.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
COMMON="--cpu-frames 0 --worst-frames 0 --scale-ref-steps 0 --exact-steps 0"
for r in 1 2; do
  for cfg in C5 C4 C3; do for kp in 1 0; do
    st=60; [ $cfg = C5 ] && st=200
    timeout -k 10 300 python -u bench.py --config $cfg --steps $st --warmup 10 $COMMON --multi-sweep none --keep-prop $kp > gpurun_out/kp_${cfg}_$kp.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/kp_${cfg}_$kp.log').read().strip().splitlines()[-1]); print('$cfg keep_prop $kp', round(d['ms_per_step']*1e3,2), 'us/frame', d['roofline']['per_kernel_avg_us'])"
  done; done
  for cfg in C2 C5; do for kp in 1 0; do
    S=32; [ $cfg = C5 ] && S=8
    timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 5 $COMMON --multi-sweep $S --multi-groups 2 --multi-steps 60 --keep-prop $kp > gpurun_out/kpm_${cfg}_$kp.log 2>&1 || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/kpm_${cfg}_$kp.log').read().strip().splitlines()[-1])
print('$cfg x $S G2 keep_prop $kp', ' | '.join(f\"{p['ms_per_batch']*1e3:.1f}us/batch {p['frac']}\" for p in d['multi_stream']['points']))"
  done; done
done
