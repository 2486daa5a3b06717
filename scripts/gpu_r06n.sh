#!/bin/bash
# Round 6 (n): final measurement of the tree: the PMC passes bench.py reads (refreshed into profiles/ on the box
# before the bench runs), the driver's bench command without the profiler, its rocprofv3 kernel trace, the trace check
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
bash scripts/pmc_lines.sh C2 C3 C4 C5 || exit 1
for c in c2:100000 c3:1000000 c4:10000000 c5:1000000; do
  cp gpurun_out/pmc_${c%%:*}.json profiles/pmc_${c%%:*}_n${c##*:}.json || exit 1
  cp gpurun_out/pmc_${c%%:*}.json gpurun_out/r06/pmc_${c%%:*}_n${c##*:}.json || exit 1
done
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/bench_driver_n.log 2>&1 || { tail -20 gpurun_out/r06/bench_driver_n.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06/bench_driver_n.log').read().splitlines() if l.startswith('{')][-1])
r=d['roofline']; print('line', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,3), 'G; avg_us', r['avg_us'], 'frac', r['frac'], 'issue', (r.get('issue') or {}).get('issue_frac'))"
rm -rf gpurun_out/r06/trace_n
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/trace_n -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/trace_n.log 2>&1 || { tail -20 gpurun_out/r06/trace_n.log; exit 1; }
d=$(dirname $(find gpurun_out/r06/trace_n -name run_kernel_trace.csv | head -1))
python3 scripts/trace_check.py $d gpurun_out/r06/trace_n.log --untraced gpurun_out/r06/bench_driver_n.log | tee gpurun_out/r06/trace_check_n.txt
python3 scripts/trace_summary.py $d 14 > gpurun_out/r06/trace_summary_n.txt
cp $d/run_kernel_stats.csv gpurun_out/r06/trace_n_kernel_stats.csv
head -20 gpurun_out/r06/trace_summary_n.txt
