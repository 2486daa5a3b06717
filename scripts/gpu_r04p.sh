#!/bin/bash
# Round 4: A/B of the instruction cuts (base = ad3a3cc, before them; w7 = current with the kept-set k_resample floor
# at 7 waves per SIMD, no SGPR spills; nostore = a timing probe without the packed pass's weight / partial stores
# (records differ by design); new = in-tree, floor 8) on C4 / C2, records compared; then the C4 PMC passes and the
# driver's bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
AB_LIBS="base=ab/libpfmpe_base.so w7=ab/libpfmpe_w7.so nostore=ab/libpfmpe_nostore.so new=" AB_CONFIGS="C4 C2" bash scripts/ab_libs.sh 2>&1 | tee gpurun_out/r04p_ab.txt || exit 1
bash scripts/pmc.sh r04p_c4 --config C4 --steps 20 --warmup 3 --worst-frames 0 --multi-sweep none --single-points none \
  --scale-ref-steps 0 --exact-steps 0 > gpurun_out/pmc_r04p_c4.txt 2>&1 || { tail -20 gpurun_out/pmc_r04p_c4.txt; exit 1; }
grep -E "^k_|VALU|FETCH|WRITE|HBM|per " gpurun_out/pmc_r04p_c4.txt | sed -n "1,40p"
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04p_driver.log 2>&1 || { tail -5 gpurun_out/r04p_driver.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04p_driver.log').read().strip().splitlines()[-1])
print('driver', round(d['ms_per_step']*1e3,2), 'us', round(d['value']/1e9,3), 'G', d['roofline']['frac'], d['roofline']['per_kernel_avg_us'])
for k, v in (d.get('single_stream') or {}).items(): print(' ', k, round(v['ms_per_frame']*1e3,1), 'us', round(v['value']/1e9,2), 'G', v['frame_frac'], v['per_kernel_avg_us'])
print(' ', [(p['config'], p['streams'], p['groups'], round(p['updates_per_s']/1e9,2), p['frac']) for p in d['multi_stream']['points']][-4:])"
