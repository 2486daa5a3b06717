#!/bin/bash
# Round 4: the top's K_total through count_targets_wave (measured neutral, reverted).  Base (5c83a80 build) vs in-tree on C2 (two
# alternating rounds of 400 frames, records compared) and the driver's command once per build, the C2 phase
# timeline of the new build, the frame shapes' identity, then the whole -m gpu suite + smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
AB_LIBS="base=ab/libpfmpe_base.so new=" AB_CONFIGS="C2 C4" bash scripts/ab_libs.sh 2>&1 | tee gpurun_out/r04zg_ab.txt || exit 1
for v in base new base new; do
  if [ $v = base ]; then export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_base.so; else unset PFMPE_LIB_OVERRIDE; fi
  timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 --single-points none --multi-sweep none > gpurun_out/r04zg_drv_$v.log 2>&1 || { tail -5 gpurun_out/r04zg_drv_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04zg_drv_$v.log').read().strip().splitlines()[-1])
print('$v driver', round(d['ms_per_step']*1e3,2), 'us', round(d['value']/1e9,3), 'G', d['roofline']['per_kernel_avg_us'])" | tee -a gpurun_out/r04zg_ab.txt
done
unset PFMPE_LIB_OVERRIDE
timeout -k 10 240 python -u scripts/diag_stamps.py 100000 > gpurun_out/r04zg_stamps_c2.log 2>&1 || { tail -5 gpurun_out/r04zg_stamps_c2.log; exit 1; }
head -12 gpurun_out/r04zg_stamps_c2.log
common="--steps 8 --warmup 0 --config C5 --particles 20000 --cpu-frames 0 --worst-frames 0 --no-timing --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for fu in 0 1 2; do
  timeout -k 10 200 python -u bench.py --gpus 1 --stream-id 0 --fused $fu --dump-records gpurun_out/zg_f$fu $common > gpurun_out/zg_f$fu.log 2>&1 || { tail -5 gpurun_out/zg_f$fu.log; exit 1; }
done
python3 - <<'PY' || exit 1
import json, sys
r = {f: json.load(open(f"gpurun_out/zg_f{f}.0.json")) for f in (0, 1, 2)}
ok = all(r[f]["records"] == r[2]["records"] and r[f]["post_sha1"] == r[2]["post_sha1"] for f in (0, 1))
print("shapes identical:", ok)
sys.exit(0 if ok else 1)
PY
bash scripts/gpu_suite.sh
