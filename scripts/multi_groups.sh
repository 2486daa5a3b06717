set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --cpu-frames 0 --worst-frames 0 --steps 100 --multi-sweep 4,8,16,32 --multi-groups 1,2,4 --multi-steps 100 > gpurun_out/mg_c2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config C5 --cpu-frames 0 --worst-frames 0 --steps 50 --multi-sweep 4,8 --multi-groups 1,2,4 --multi-steps 50 > gpurun_out/mg_c5.log 2>&1
rc=$?
for c in c2 c5; do python3 -c "
import json; d=json.loads(open('gpurun_out/mg_$c.log').read().strip().splitlines()[-1])
print('$c', round(d['value']/1e9,3), d.get('scaling_reference'))
for p in d['multi_stream']['points']: print('  S', p['streams'], 'G', p['groups'], round(p['updates_per_s']/1e9,2), 'G/s', p['frac'], round(p['ms_per_batch']*1e3,1), 'us/batch')
"; done
exit $rc
