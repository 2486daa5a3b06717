#!/bin/bash
# Round-2 re-entry pass from the rebuilt tree: the whole -m gpu suite, smoke, the default bench line and
# C3 / C4 / C5 lines.  Every GPU step has its own time limit; steps are chained with && (stop at the first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
t=${TAG:-r02g}
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/${t}_gpu_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${t}_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/${t}_bench_c2.log 2>&1 &&
timeout -k 10 200 python -u bench.py --config C4 --cpu-frames 0 --steps 60 --warmup 6 --worst-frames 0 > gpurun_out/${t}_bench_c4.log 2>&1 &&
timeout -k 10 200 python -u bench.py --config C3 --cpu-frames 0 --steps 60 --warmup 6 --worst-frames 0 > gpurun_out/${t}_bench_c3.log 2>&1 &&
timeout -k 10 200 python -u bench.py --config C5 --cpu-frames 0 --steps 100 --warmup 10 --worst-frames 0 > gpurun_out/${t}_bench_c5.log 2>&1
rc=$?
tail -3 gpurun_out/${t}_gpu_tests.log
for c in c2 c4 c3 c5; do python3 -c "import json; d=json.load(open('gpurun_out/${t}_bench_$c.log')); print('$c', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,3), 'G/s', d['roofline']['per_kernel_avg_us'], d['roofline']['frac'])" 2>/dev/null; done
exit $rc
