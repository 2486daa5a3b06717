#!/bin/bash
# Round 4: (1) issue cost of the instructions the weighing / resampling kernels are made of (scripts/isa_rates.hip);
# (2) the merged k_group_top_wide launch: the frame-shape / count / batched tests, then C4 A/B against the split
# launches (diag 32768 = DIAG_SPLIT_TOP), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 ./scripts/isa_rates.bin > gpurun_out/r04m_isa_rates.txt 2>&1 || { cat gpurun_out/r04m_isa_rates.txt; exit 1; }
cat gpurun_out/r04m_isa_rates.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_frame_shapes.py \
  tests/test_gpu_resample_counts.py tests/test_gpu_multi.py tests/test_gpu_defer.py > gpurun_out/r04m_tests.log 2>&1 \
  || { tail -30 gpurun_out/r04m_tests.log; exit 1; }
tail -2 gpurun_out/r04m_tests.log
for rep in 1 2; do
  for d in 0 32768; do
    timeout -k 10 300 python -u bench.py --config C4 --steps 40 --warmup 5 --cpu-frames 0 --worst-frames 0 \
      --multi-sweep 2 --multi-groups 1 --multi-steps 20 --scale-ref-steps 0 --exact-steps 0 --single-points none \
      --diag $d > gpurun_out/r04m_c4_${d}_$rep.log 2>&1 || { tail -5 gpurun_out/r04m_c4_${d}_$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04m_c4_${d}_$rep.log').read().strip().splitlines()[-1])
print('diag $d C4', round(d['ms_per_step']*1e3,1), 'us', round(d['value']/1e9,2), 'G', d['roofline']['per_kernel_avg_us'], '|',
      [(p['streams'], round(p['updates_per_s']/1e9,2), round(p['ms_per_batch']*1e3,1)) for p in d['multi_stream']['points']])"
  done
done
