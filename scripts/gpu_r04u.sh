#!/bin/bash
# Round 4 closing measurements: PMC passes of C2 / C4 / C5 (the bench's traffic sources, profiles/pmc_<cfg>_n<N>.json),
# the driver's bench command three times, and its rocprofv3 kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
common="--steps 20 --warmup 3 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
bash scripts/pmc.sh c2_n100000 $common > gpurun_out/pmc_u_c2.txt 2>&1 || { tail -20 gpurun_out/pmc_u_c2.txt; exit 1; }
bash scripts/pmc.sh c4_n10000000 --config C4 $common > gpurun_out/pmc_u_c4.txt 2>&1 || { tail -20 gpurun_out/pmc_u_c4.txt; exit 1; }
bash scripts/pmc.sh c5_n1000000 --config C5 $common > gpurun_out/pmc_u_c5.txt 2>&1 || { tail -20 gpurun_out/pmc_u_c5.txt; exit 1; }
echo "pmc done"
for rep in 1 2 3; do
  timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04u_bench_$rep.log 2>&1 || { tail -5 gpurun_out/r04u_bench_$rep.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04u_bench_$rep.log').read().strip().splitlines()[-1])
print('driver', round(d['ms_per_step']*1e3,2), 'us', round(d['value']/1e9,3), 'G', d['roofline']['frac'], d['roofline']['per_kernel_avg_us'], d['roofline']['launches_timed'])
for k, v in (d.get('single_stream') or {}).items(): print(' ', k, round(v['ms_per_frame']*1e3,1), 'us', round(v['value']/1e9,2), 'G', v['frame_frac'], v['per_kernel_avg_us'])
print(' ', [(p['config'], p['streams'], p['groups'], round(p['updates_per_s']/1e9,2), p['frac']) for p in d['multi_stream']['points']][-4:])"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04u_trace -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04u_trace.log 2>&1 || { tail -5 gpurun_out/r04u_trace.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r04u_trace/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(f"{r['Name'][:70]:70s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:9.2f} us")
PY
