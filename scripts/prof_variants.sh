#!/bin/bash
# rocprofv3 kernel traces of bench variants: prof_variants.sh <tag>:<bench args> ...
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for spec in "$@"; do
  tag=${spec%%:*}; args=${spec#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pv_$tag -o run --output-format csv -- python3 bench.py --cpu-frames 0 --no-timing $args > gpurun_out/pv_$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/pv_$tag.log; exit $rc; fi
  python3 scripts/trace_summary.py gpurun_out/pv_$tag 4 | head -3
done
