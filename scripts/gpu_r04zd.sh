#!/bin/bash
# Round 4: k_weigh_stream's occupancy floor for the wide-marker instances (MAXM > 5, C3's 12 markers): base
# (6 waves, 33 VGPRs spilled to scratch), wide5 (5 waves) and in-tree (4 waves, no spills) on C3, two alternating
# rounds, records compared; then the frame shapes' identity and the whole -m gpu suite + smoke on the in-tree build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
AB_LIBS="base=ab/libpfmpe_base.so wide5=ab/libpfmpe_wide5.so new=" AB_CONFIGS="C3" bash scripts/ab_libs.sh 2>&1 | tee gpurun_out/r04zd_ab.txt || exit 1
common="--steps 8 --warmup 0 --config C5 --particles 20000 --cpu-frames 0 --worst-frames 0 --no-timing --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for fu in 0 1 2; do
  timeout -k 10 200 python -u bench.py --gpus 1 --stream-id 0 --fused $fu --dump-records gpurun_out/zd_f$fu $common > gpurun_out/zd_f$fu.log 2>&1 || { tail -5 gpurun_out/zd_f$fu.log; exit 1; }
done
python3 - <<'PY' || exit 1
import json, sys
r = {f: json.load(open(f"gpurun_out/zd_f{f}.0.json")) for f in (0, 1, 2)}
ok = all(r[f]["records"] == r[2]["records"] and r[f]["post_sha1"] == r[2]["post_sha1"] for f in (0, 1))
print("shapes identical:", ok)
sys.exit(0 if ok else 1)
PY
bash scripts/gpu_suite.sh
