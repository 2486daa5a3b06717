#!/bin/bash
# A/B of the batched path (pfmpe_step_multi) against ab/libpfmpe_base.so: C2 streams, S = 16 and 32, one and two
# concurrent batches, alternating libraries.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_base.so; else unset PFMPE_LIB_OVERRIDE; fi
    timeout -k 10 300 python -u bench.py --config C2 --steps 20 --warmup 5 --cpu-frames 0 --worst-frames 0 --scale-ref-steps 0 \
      --exact-steps 0 --multi-sweep ${AB_SWEEP:-16,32} --multi-groups 1,2 --multi-steps 100 > gpurun_out/abm_$v.log 2>&1 || { tail gpurun_out/abm_$v.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/abm_$v.log').read().strip().splitlines()[-1])
print('$v', ' | '.join(f\"S{p['streams']}G{p['groups']} {p['ms_per_batch']*1e3:.1f}us {p['frac']}\" for p in d['multi_stream']['points']))"
  done
done
