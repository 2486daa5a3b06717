#!/bin/bash
# A/B of the in-tree library (base) against a variant build ($VARIANT, same ABI) over configs, alternating;
# each bench time-limited; stop on the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for cfg in ${CONFIGS:-C4 C3 C5}; do
  st=60; [ $cfg = C2 ] && st=400
  for r in 1 2 3; do
    for v in base var; do
      if [ $v = var ]; then export PFMPE_LIB_OVERRIDE=$PWD/$VARIANT; else unset PFMPE_LIB_OVERRIDE; fi
      timeout -k 10 300 python bench.py --config $cfg --cpu-frames 0 --steps $st --warmup 5 --worst-frames 0 \
        ${AB_MULTI:---multi-sweep 1 --multi-groups 1 --multi-steps 5} --scale-ref-steps 0 --diag ${AB_DIAG:-0} > gpurun_out/abv_$v.log 2>&1 || { tail gpurun_out/abv_$v.log; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/abv_$v.log')); print('$cfg $v', round(d['ms_per_step']*1e3,2), 'us/frame', d['roofline']['per_kernel_avg_us'], [(p['streams'], p['groups'], round(p['updates_per_s']/1e9,2)) for p in (d.get('multi_stream') or {}).get('points', []) if p['streams'] > 1])"
    done
  done
done
unset PFMPE_LIB_OVERRIDE
