#!/bin/bash
# Round 6 (k): the driver's exact bench command, its rocprofv3 kernel trace and the trace check
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/bench_driver_k.log 2>&1 || { tail -20 gpurun_out/r06/bench_driver_k.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06/bench_driver_k.log').read().splitlines() if l.startswith('{')][-1])
r=d['roofline']; print('line', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,3), 'G; avg_us', r['avg_us'], 'frac', r['frac'], 'issue', (r.get('issue') or {}).get('issue_frac'))"
rm -rf gpurun_out/r06/trace_k
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/trace_k -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/trace_k.log 2>&1 || { tail -20 gpurun_out/r06/trace_k.log; exit 1; }
d=$(dirname $(find gpurun_out/r06/trace_k -name run_kernel_trace.csv | head -1))
python3 scripts/trace_check.py $d gpurun_out/r06/trace_k.log | tee gpurun_out/r06/trace_check_k.txt
python3 scripts/trace_summary.py $d 12 > gpurun_out/r06/trace_summary_k.txt
head -30 gpurun_out/r06/trace_summary_k.txt
