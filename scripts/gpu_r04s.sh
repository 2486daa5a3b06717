#!/bin/bash
# Round 4: the scalar block-boundary count with its sign-extension fix (the bug broke the shapes' identity, r04r): the shapes'
# records on C5 N=20000 (fused 0 / 1 / 2) first, then the whole -m gpu suite + smoke, then C4 / C5 frames.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
common="--steps 8 --warmup 0 --config C5 --particles 20000 --cpu-frames 0 --worst-frames 0 --no-timing --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for fu in 0 1 2; do
  timeout -k 10 200 python -u bench.py --gpus 1 --stream-id 0 --fused $fu --dump-records gpurun_out/s_f$fu $common > gpurun_out/s_f$fu.log 2>&1 || { tail -5 gpurun_out/s_f$fu.log; exit 1; }
done
python3 - <<'PY' || exit 1
import json, sys
r = {f: json.load(open(f"gpurun_out/s_f{f}.0.json")) for f in (0, 1, 2)}
ok = all(r[f]["records"] == r[2]["records"] and r[f]["post_sha1"] == r[2]["post_sha1"] for f in (0, 1))
print("shapes identical:", ok)
sys.exit(0 if ok else 1)
PY
bash scripts/gpu_suite.sh || exit 1
for c in C4 C5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 40 --warmup 5 --cpu-frames 0 --worst-frames 0 \
    --multi-sweep $([ $c = C4 ] && echo 2 || echo 32) --multi-groups $([ $c = C4 ] && echo 1 || echo 2) --multi-steps 20 \
    --scale-ref-steps 0 --exact-steps 0 --single-points none > gpurun_out/r04s_$c.log 2>&1 || { tail -5 gpurun_out/r04s_$c.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04s_$c.log').read().strip().splitlines()[-1])
print('$c', round(d['ms_per_step']*1e3,1), 'us', round(d['value']/1e9,2), 'G', d['roofline']['per_kernel_avg_us'], '|',
      [(p['streams'], p['groups'], round(p['updates_per_s']/1e9,2), p['frac'], round(p['ms_per_batch']*1e3,1)) for p in d['multi_stream']['points']])"
done
