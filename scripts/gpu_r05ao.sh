#!/bin/bash
# Round 5 (ao): the final tree: the whole -m gpu suite + smoke, the driver's default bench line, the C2 kernel trace
# of the same line's shape, and the C2 PMC passes (profiles/pmc_c2_n100000.json)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_suite.sh || exit 1
timeout -k 10 900 python -u bench.py > gpurun_out/r05ao_bench.log 2>&1 || { tail -5 gpurun_out/r05ao_bench.log; exit 1; }
tail -c 400 gpurun_out/r05ao_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05ao_prof -o run --output-format csv -- python3 bench.py --cpu-frames 0 --worst-frames 0 --multi-sweep none --scale-ref-steps 0 --exact-steps 0 > gpurun_out/r05ao_prof.log 2>&1 || { tail -5 gpurun_out/r05ao_prof.log; exit 1; }
python3 scripts/trace_summary.py gpurun_out/r05ao_prof 6 > gpurun_out/r05ao_trace_summary.txt 2>&1; head -8 gpurun_out/r05ao_trace_summary.txt
bash scripts/pmc_lines.sh C2 || exit 1
cat gpurun_out/pmcl_c2.txt | head -30
