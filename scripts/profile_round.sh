#!/bin/bash
# Round profile: bench (with cpu_baseline), rocprofv3 kernel-trace stats of the same command, one per
# config given (default C2).  Each GPU step has its own time limit; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${TAG:-r01}
for cfg in ${CONFIGS:-C2}; do
  lc=$(echo $cfg | tr A-Z a-z)
  extra=""; [ "$cfg" != "C2" ] && extra="--cpu-frames 0 --steps ${STEPS:-50} --warmup 5"
  timeout -k 10 600 python bench.py --config $cfg $extra > gpurun_out/${tag}_${lc}_bench.log 2>&1 || { tail gpurun_out/${tag}_${lc}_bench.log; exit 1; }
  cat gpurun_out/${tag}_${lc}_bench.log
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_${lc}_prof -o run --output-format csv -- python3 bench.py --config $cfg --cpu-frames 0 --no-timing ${extra/--cpu-frames 0/} > gpurun_out/${tag}_${lc}_prof.log 2>&1 || { tail gpurun_out/${tag}_${lc}_prof.log; exit 1; }
  python3 scripts/trace_summary.py gpurun_out/${tag}_${lc}_prof > gpurun_out/${tag}_${lc}_trace_summary.txt 2>&1
  head -4 gpurun_out/${tag}_${lc}_trace_summary.txt
done
