#!/bin/bash
# Round 4 close, final tree: the C2 (k_frame2) phase timeline, the driver's bench command three times and the
# rocprofv3 kernel trace of that command.  Logs under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/diag_stamps.py 100000 > gpurun_out/r04y_stamps_c2.log 2>&1 \
  || { tail -5 gpurun_out/r04y_stamps_c2.log; exit 1; }
cat gpurun_out/r04y_stamps_c2.log
for rep in 1 2 3; do
  timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04y_bench_$rep.log 2>&1 || { tail -5 gpurun_out/r04y_bench_$rep.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04y_bench_$rep.log').read().strip().splitlines()[-1])
print('driver', round(d['ms_per_step']*1e3,2), 'us', round(d['value']/1e9,3), 'G', d['roofline']['frac'], d['roofline']['per_kernel_avg_us'], d['roofline']['launches_timed'])
for k, v in (d.get('single_stream') or {}).items(): print(' ', k, round(v['ms_per_frame']*1e3,1), 'us', round(v['value']/1e9,2), 'G', v['frame_frac'], v['per_kernel_avg_us'])
print(' ', [(p['config'], p['streams'], p['groups'], round(p['updates_per_s']/1e9,2), p['frac']) for p in d['multi_stream']['points']][-4:])"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04y_trace -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04y_trace.log 2>&1 || { tail -5 gpurun_out/r04y_trace.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r04y_trace/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:10]:
    print(f"{r['Name'][:70]:70s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:9.2f} us")
PY
