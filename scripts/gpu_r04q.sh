#!/bin/bash
# Round 4 debug: test_bench_dist's records differ between the 2-rank (one shared GPU) and 1-rank runs of C5 N=20000.
# Records of the same stream under each frame shape (fused 0 / 1 / 2), and the 2-rank run, compared field by field.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
common="--steps 6 --warmup 2 --config C5 --particles 20000 --cpu-frames 0 --worst-frames 0 --no-timing --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for fu in 0 1 2; do
  timeout -k 10 200 python -u bench.py --gpus 1 --stream-id 0 --fused $fu --dump-records gpurun_out/q_f$fu $common > gpurun_out/q_f$fu.log 2>&1 || { tail -5 gpurun_out/q_f$fu.log; exit 1; }
done
PFMPE_BENCH_DEVICE=0 MASTER_ADDR=127.0.0.1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --dump-records gpurun_out/q_two $common > gpurun_out/q_two.log 2>&1 || { tail -5 gpurun_out/q_two.log; exit 1; }
python3 - <<'PY'
import json
def load(p): return json.load(open(p))
runs = {f"fused{f}": load(f"gpurun_out/q_f{f}.0.json") for f in (0, 1, 2)}
runs["two_rank0"] = load("gpurun_out/q_two.0.json")
base = runs["fused2"]
for name, r in runs.items():
    diffs = []
    for i, (a, b) in enumerate(zip(base["records"], r["records"])):
        d = {k: (a[k], b[k]) for k in a if a[k] != b[k] and k not in ("winner_pose", "most_likely_pose")}
        if a["winner_pose"] != b["winner_pose"]: d["winner_pose"] = "differs"
        if d: diffs.append((i, d))
    print(name, "post_sha1 equal" if r["post_sha1"] == base["post_sha1"] else "post_sha1 DIFFERS", "| frames differing:", len(diffs))
    for i, d in diffs[:3]:
        print("   frame", i, {k: v for k, v in list(d.items())[:8]})
PY
grep -h "shape\|weigh_pass" gpurun_out/q_f*.log gpurun_out/q_two.log | cut -c1-200 | sed -n "1,12p"
