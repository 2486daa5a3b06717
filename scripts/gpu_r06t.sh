#!/bin/bash
# Round 6 (t): the driver's bench command three times on the final tree (box-to-run spread of the line)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/bench_final_x3_$i.log 2>&1 || { tail -20 gpurun_out/r06/bench_final_x3_$i.log; exit 1; }
  python3 - gpurun_out/r06/bench_final_x3_$i.log <<'PY' | tee -a gpurun_out/r06/bench_final_x3.txt
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith('{"metric"')][-1])
r = d["roofline"]; ss = d["single_stream"]
ms = {f"{p['streams']}x{p['config']}/{p['groups']}": round(p["updates_per_s"] / 1e9, 2) for p in d["multi_stream"]["points"] if p["streams"] in (2, 32) or p["config"] != "C2"}
print(f"C2 {d['ms_per_step']*1e3:.2f} us {d['value']/1e9:.3f} G k_frame2 {r['avg_us']} us frac {r['frac']} issue {r['issue']['issue_frac']}; "
      f"C3 {ss['C3']['ms_per_frame']*1e3:.1f} us, C4 {ss['C4']['ms_per_frame']*1e3:.1f} us, C5 {d['scaling_reference']['ms_per_frame']*1e3:.1f} us; multi G {ms}")
PY
done
