#!/bin/bash
# A/B of the in-tree library against ab/libpfmpe_base.so (built from an earlier commit): alternating
# short benches, then the phase stamps of the in-tree k_frame2.  Each step time-limited; stop on failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
ARGS=${AB_ARGS:---cpu-frames 0 --steps 400 --warmup 40}
for r in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_base.so; else unset PFMPE_LIB_OVERRIDE; fi
    timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab_$v.log 2>&1 || { tail gpurun_out/ab_$v.log; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.log')); print('$v', round(d['ms_per_step']*1e3,2), 'us/frame', d['roofline']['per_kernel_avg_us'])"
  done
done
unset PFMPE_LIB_OVERRIDE
PFMPE_FUSED=2 timeout -k 10 300 python scripts/diag_stamps.py ${STAMP_N:-100000} > gpurun_out/stamps.log 2>&1 || { cat gpurun_out/stamps.log; exit 1; }
cat gpurun_out/stamps.log
