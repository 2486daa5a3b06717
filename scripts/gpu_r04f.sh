#!/bin/bash
# Round 4 A/B: (1) k_weigh_pk at a 5-wave floor (96 VGPRs, libpfmpe_pk5.so) against the compiler's choice
# (125 VGPRs, 4 waves) at C4 / C5; (2) where the packed pass stops paying: fp32 streams of 1M-4M particles with the
# packed pass (default) and without it (PFMPE_DIAG 4096).  Alternating, two rounds.  Logs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=pf_monocular_pose_estimator_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_weigh_pk.py tests/test_gpu_multi.py -k "pk or streaming" -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04f_tests.log 2>&1 || { tail -20 gpurun_out/r04f_tests.log; exit 1; }
tail -2 gpurun_out/r04f_tests.log
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --cpu-frames 0 --worst-frames 0 --multi-sweep none \
    --single-points none "$@" > gpurun_out/r04f_$tag.log 2>&1 || { tail -5 gpurun_out/r04f_$tag.log; return 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04f_$tag.log').read().strip().splitlines()[-1])
print('$tag', round(d['ms_per_step']*1e3,1), 'us/frame', round(d['value']/1e9,2), 'G/s', d['roofline'].get('per_kernel_avg_us'))"
}
for rep in 1 2; do
  for c in C4 C5; do
    run ${c}_w4_$rep --config $c || exit 1
    PFMPE_LIB_OVERRIDE=$PWD/$L/libpfmpe_pk5.so run ${c}_w5_$rep --config $c || exit 1
  done
  for n in 1000000 2000000 4000000; do
    run C5n${n}_pk_$rep --config C5 --particles $n || exit 1
    run C5n${n}_nopk_$rep --config C5 --particles $n --diag 4096 || exit 1
  done
done
