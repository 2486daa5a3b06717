#!/bin/bash
# Round 4 close, after the marker phases: the C2 (k_frame2) phase timeline, the driver's bench command three
# times, the C4 instruction-count PMC pass and the rocprofv3 kernel trace of the driver's command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/diag_stamps.py 100000 > gpurun_out/r04zc_stamps_c2.log 2>&1 \
  || { tail -5 gpurun_out/r04zc_stamps_c2.log; exit 1; }
cat gpurun_out/r04zc_stamps_c2.log
for rep in 1 2 3; do
  timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04zc_bench_$rep.log 2>&1 || { tail -5 gpurun_out/r04zc_bench_$rep.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04zc_bench_$rep.log').read().strip().splitlines()[-1])
print('driver', round(d['ms_per_step']*1e3,2), 'us', round(d['value']/1e9,3), 'G', d['roofline']['frac'], d['roofline']['per_kernel_avg_us'], d['roofline']['launches_timed'])
for k, v in (d.get('single_stream') or {}).items(): print(' ', k, round(v['ms_per_frame']*1e3,1), 'us', round(v['value']/1e9,2), 'G', v['frame_frac'], v['per_kernel_avg_us'])
print(' ', [(p['config'], p['streams'], p['groups'], round(p['updates_per_s']/1e9,2), p['frac']) for p in d['multi_stream']['points']][-4:])"
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVE_CYCLES \
  --output-format csv -d gpurun_out/r04zc_pmc -o run -- python3 bench.py --config C4 --cpu-frames 0 --no-timing --steps 20 --warmup 3 \
  --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0 > gpurun_out/r04zc_pmc.log 2>&1 \
  || { tail -5 gpurun_out/r04zc_pmc.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/r04zc_pmc > gpurun_out/r04zc_pmc.txt 2>&1 || true
grep -A9 -E "^k_(resample|weigh_pk)$" gpurun_out/r04zc_pmc.txt | sed -n "1,30p"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04zc_trace -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04zc_trace.log 2>&1 || { tail -5 gpurun_out/r04zc_trace.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r04zc_trace/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:10]:
    print(f"{r['Name'][:70]:70s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:9.2f} us")
PY
