#!/bin/bash
# Round 4: where the C2 frame's time outside k_frame2 goes.  A HIP API + kernel trace of the driver's bench command
# (no counters), summarised per API call and as the gap between consecutive k_frame2 dispatches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d gpurun_out/r04g_trace -o run -- \
  python3 bench.py --steps 200 --warmup 20 --cpu-frames 0 --worst-frames 0 --scale-ref-steps 0 --exact-steps 0 \
  --multi-sweep none --single-points none --no-timing > gpurun_out/r04g_trace.log 2>&1 || { tail -5 gpurun_out/r04g_trace.log; exit 1; }
tail -1 gpurun_out/r04g_trace.log | cut -c1-300
python3 - <<'PY'
import csv, glob, collections
d = "gpurun_out/r04g_trace"
kt = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))
ht = sorted(glob.glob(f"{d}/**/*hip_api_trace.csv", recursive=True))
ks = [r for r in csv.DictReader(open(kt[0])) if "k_frame2" in r["Kernel_Name"]]
ks.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ks]
gap = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(ks, ks[1:])]
per = [(int(b["Start_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3 for a, b in zip(ks, ks[1:])]
def q(v):
    v = sorted(v); n = len(v)
    return f"n={n} median {v[n//2]:.2f} p10 {v[n//10]:.2f} p90 {v[9*n//10]:.2f} mean {sum(v)/n:.2f}"
print("k_frame2 duration us:", q(dur))
print("gap end->next start us:", q(gap))
print("start->next start us:", q(per))
if ht:
    acc = collections.defaultdict(list)
    rows = list(csv.DictReader(open(ht[0])))
    for r in rows:
        acc[r["Function"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for f, v in sorted(acc.items(), key=lambda kv: -sum(kv[1]))[:12]:
        print(f"{f:40s} {q(v)}")
    # launch call -> kernel start latency for k_frame2 (matched by correlation id)
    launches = {r["Correlation_Id"]: r for r in rows if "Launch" in r["Function"]}
    lat = []
    for k in ks:
        l = launches.get(k.get("Correlation_Id"))
        if l:
            lat.append((int(k["Start_Timestamp"]) - int(l["Start_Timestamp"])) / 1e3)
    if lat:
        print("launch call start -> kernel start us:", q(lat))
PY
