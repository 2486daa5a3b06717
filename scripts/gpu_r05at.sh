#!/bin/bash
# Round 5 (at): the driver's default bench line with the longer 2 x C4 batch point
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > gpurun_out/r05at_bench.log 2>&1 || { tail -5 gpurun_out/r05at_bench.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open('gpurun_out/r05at_bench.log').read().strip().splitlines()[-1])
print('C2', round(d['ms_per_step'] * 1e3, 2), 'us', round(d['value'] / 1e9, 3), 'G')
for k, v in d['single_stream'].items(): print(k, round(v['ms_per_frame'] * 1e3, 2), 'us', round(v['value'] / 1e9, 2), 'G')
for p in d['multi_stream']['points'][-3:]: print(p['streams'], 'x', p['config'], p['groups'], round(p['ms_per_batch'] * 1e3, 1), 'us', round(p['updates_per_s'] / 1e9, 2), 'G', p['frac'])
PY
