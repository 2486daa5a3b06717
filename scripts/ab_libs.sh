#!/bin/bash
# A/B/C... of several builds of the library on one box: AB_LIBS="name=path ..." (the in-tree build is "new"),
# configs AB_CONFIGS (default C4 C5), two alternating rounds each; frame records compared against the first lib.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
COMMON="--cpu-frames 0 --worst-frames 0 --multi-sweep none --scale-ref-steps 0 --exact-steps 0"
LIBS=${AB_LIBS:-"base=ab/libpfmpe_base.so new="}
for cfg in ${AB_CONFIGS:-C4 C5}; do
  case $cfg in C2) st=400;; C5) st=200;; *) st=60;; esac
  for r in 1 2; do
    for lv in $LIBS; do
      v=${lv%%=*}; p=${lv#*=}
      if [ -n "$p" ]; then export PFMPE_LIB_OVERRIDE=$PWD/$p; else unset PFMPE_LIB_OVERRIDE; fi
      timeout -k 10 300 python -u bench.py --config $cfg --steps $st --warmup 20 $COMMON --dump-records gpurun_out/rec_${cfg}_$v \
        > gpurun_out/abl_${cfg}_$v.log 2>&1 || { tail gpurun_out/abl_${cfg}_$v.log; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/abl_${cfg}_$v.log').read().strip().splitlines()[-1]); print('$cfg', '$v', round(d['ms_per_step']*1e3,2), 'us/frame', d['roofline']['per_kernel_avg_us'])"
    done
  done
  unset PFMPE_LIB_OVERRIDE
  first=""
  for lv in $LIBS; do
    v=${lv%%=*}
    if [ -z "$first" ]; then first=$v; continue; fi
    if cmp -s gpurun_out/rec_${cfg}_$first.0.json gpurun_out/rec_${cfg}_$v.0.json; then echo "$cfg $v records identical to $first"; else echo "$cfg $v RECORDS DIFFER from $first"; fi
  done
done
