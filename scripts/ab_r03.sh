#!/bin/bash
# A/B of the in-tree library against ab/libpfmpe_base.so on C2 / C5 / C4 (alternating, two rounds each), with
# the frame records of both dumped and compared (the changes under test must be bit-identical).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
COMMON="--cpu-frames 0 --worst-frames 0 --multi-sweep none --scale-ref-steps 0"
for cfg in ${AB_CONFIGS:-C2 C5 C4}; do
  case $cfg in C2) st=400;; C5) st=200;; *) st=60;; esac
  for r in 1 2; do
    for v in base new; do
      if [ $v = base ]; then export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_base.so; else unset PFMPE_LIB_OVERRIDE; fi
      timeout -k 10 300 python -u bench.py --config $cfg --steps $st --warmup 20 $COMMON --dump-records gpurun_out/rec_${cfg}_$v \
        > gpurun_out/ab_${cfg}_$v.log 2>&1 || { tail gpurun_out/ab_${cfg}_$v.log; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/ab_${cfg}_$v.log').read().strip().splitlines()[-1]); print('$cfg', '$v', round(d['ms_per_step']*1e3,2), 'us/frame', d['roofline']['per_kernel_avg_us'])"
    done
  done
  unset PFMPE_LIB_OVERRIDE
  if cmp -s gpurun_out/rec_${cfg}_base.0.json gpurun_out/rec_${cfg}_new.0.json; then echo "$cfg records identical"; else echo "$cfg RECORDS DIFFER"; fi
done
