#!/bin/bash
# Round 4 bisect: do the frame shapes (fused 0 = two launches, 1 = k_frame, 2 = k_frame2) still give identical records
# and particle sets on C5 N=20000?  For each library build: base (ad3a3cc), 1023644 (scalar block count),
# ea45682 (band guard, div_by_S, fixed-point scans, folded argmax), w7 (cf2987a + 7-wave k_resample), new (in-tree).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
common="--steps 8 --warmup 0 --config C5 --particles 20000 --cpu-frames 0 --worst-frames 0 --no-timing --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for lv in base=ab/libpfmpe_base.so c1023644=ab/libpfmpe_1023644.so cea45682=ab/libpfmpe_ea45682.so w7=ab/libpfmpe_w7.so new=; do
  v=${lv%%=*}; p=${lv#*=}
  if [ -n "$p" ]; then export PFMPE_LIB_OVERRIDE=$PWD/$p; else unset PFMPE_LIB_OVERRIDE; fi
  for fu in 0 1 2; do
    timeout -k 10 200 python -u bench.py --gpus 1 --stream-id 0 --fused $fu --dump-records gpurun_out/r_${v}_f$fu $common > gpurun_out/r_${v}_f$fu.log 2>&1 || { tail -5 gpurun_out/r_${v}_f$fu.log; exit 1; }
  done
  python3 - "$v" <<'PY'
import json, sys
v = sys.argv[1]
r = {f: json.load(open(f"gpurun_out/r_{v}_f{f}.0.json")) for f in (0, 1, 2)}
def cmp(a, b):
    for i, (x, y) in enumerate(zip(a["records"], b["records"])):
        if x != y:
            return f"first differing frame {i}: " + str({k: (x[k], y[k]) for k in ("winner_idx", "prob_sum", "iters") if x[k] != y[k]})
    return "records equal" + ("" if a["post_sha1"] == b["post_sha1"] else ", post DIFFERS")
print(v, "| f0 vs f2:", cmp(r[0], r[2]), "| f1 vs f2:", cmp(r[1], r[2]))
PY
done
unset PFMPE_LIB_OVERRIDE
