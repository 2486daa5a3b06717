#!/bin/bash
# Round 6 (j): batches finished inside k_resample_owners_multi (no k_resample_final_multi): batch tests, then the
# default bench line (multi-stream points) for the new and the round-start library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_multi.py tests/test_gpu_resample_owners.py tests/test_gpu_defer.py tests/test_bench_dist.py > gpurun_out/r06/tests_j.log 2>&1 || { tail -40 gpurun_out/r06/tests_j.log; exit 1; }
tail -n 1 gpurun_out/r06/tests_j.log
for v in new r05; do
  if [ $v = new ]; then unset PFMPE_LIB_OVERRIDE; else export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_$v.so; fi
  timeout -k 10 400 python -u bench.py --cpu-frames 0 > gpurun_out/r06/bench_j_$v.log 2>&1 || { tail -5 gpurun_out/r06/bench_j_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06/bench_j_$v.log').read().splitlines() if l.startswith('{')][-1])
print('$v C2', round(d['ms_per_step']*1e3,2), 'us', round(d['value']/1e9,3), 'G')
for p in d['multi_stream']['points']: print('$v', p['config'], p['streams'], p['groups'], round(p['updates_per_s']/1e9,2), 'G', p['frac'], p.get('counter_frac'))
for k,p in (d.get('single_stream') or {}).items(): print('$v single', k, round(p['ms_per_frame']*1e3,1), 'us', p['per_kernel_avg_us'])
" | tee -a gpurun_out/r06/bench_j.txt
done
unset PFMPE_LIB_OVERRIDE
