cd "${GRAFT_REPO_ROOT:-.}"
AB_CONFIGS="C2 C5 C4 C3" bash scripts/ab_r03.sh || exit 1
for cfg in C5 C4; do for kp in 0 1; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 60 --warmup 10 --cpu-frames 0 --worst-frames 0 --multi-sweep none --scale-ref-steps 0 --keep-prop $kp > gpurun_out/kp_${cfg}_$kp.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/kp_${cfg}_$kp.log').read().strip().splitlines()[-1]); print('$cfg keep_prop $kp', round(d['ms_per_step']*1e3,2), 'us/frame', d['roofline']['per_kernel_avg_us'])"
done; done
