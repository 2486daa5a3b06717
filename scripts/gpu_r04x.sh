#!/bin/bash
# Round 4: the block boundary count through count_targets_wave too: the frame shapes' identity,
# the whole -m gpu suite + smoke, then base (ad3a3cc) vs in-tree on C4 / C5 (two alternating rounds, records compared).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
common="--steps 8 --warmup 0 --config C5 --particles 20000 --cpu-frames 0 --worst-frames 0 --no-timing --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for fu in 0 1 2; do
  timeout -k 10 200 python -u bench.py --gpus 1 --stream-id 0 --fused $fu --dump-records gpurun_out/x_f$fu $common > gpurun_out/x_f$fu.log 2>&1 || { tail -5 gpurun_out/x_f$fu.log; exit 1; }
done
python3 - <<'PY' || exit 1
import json, sys
r = {f: json.load(open(f"gpurun_out/x_f{f}.0.json")) for f in (0, 1, 2)}
ok = all(r[f]["records"] == r[2]["records"] and r[f]["post_sha1"] == r[2]["post_sha1"] for f in (0, 1))
print("shapes identical:", ok)
sys.exit(0 if ok else 1)
PY
bash scripts/gpu_suite.sh || exit 1
AB_LIBS="base=ab/libpfmpe_base.so new=" AB_CONFIGS="C4 C5" bash scripts/ab_libs.sh 2>&1 | tee gpurun_out/r04x_ab.txt || exit 1
