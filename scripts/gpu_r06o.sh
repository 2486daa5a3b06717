#!/bin/bash
# Round 6 (o): where the fused hand-off's time goes.  Diagnostic builds of the rejected PkTail variant
# (ab/libpfmpe_pkt*.so, built from the reverted patch with PFMPE_PKTAIL_DIAG / PFMPE_PKTAIL_WT): pkt0 = the full fused
# tail; pkt1 = write-through partial stores + the post-loop drain only (hand-off launches kept); pkt1p = plain stores +
# drain; pkt2 = drain + the sharded arrivals, no group reductions (launches kept).  C4 / C5 / C3 k_weigh_pk averages.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
common="--cpu-frames 0 --worst-frames 0 --multi-sweep none --single-points none --scale-ref-steps 0 --exact-steps 0"
for cfg in C4 C5 C3; do
  for v in tree pkt1p pkt1 pkt2 pkt0; do
    if [ $v = tree ]; then unset PFMPE_LIB_OVERRIDE; else export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_$v.so; fi
    timeout -k 10 200 python -u bench.py --config $cfg --steps 200 --warmup 10 $common > gpurun_out/r06/ab_o_$v.log 2>&1 || { tail -5 gpurun_out/r06/ab_o_$v.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06/ab_o_$v.log').read().splitlines() if l.startswith('{')][-1])
r=d['roofline']; print('$cfg $v', round(d['ms_per_step']*1e3,2), 'us/frame', round(d['value']/1e9,2), 'G', r['per_kernel_avg_us'])" | tee -a gpurun_out/r06/ab_o.txt
  done
done
unset PFMPE_LIB_OVERRIDE
