#!/bin/bash
# Round 4, k_weigh_pk + deferred resampling first pass: bit-identity tests of the packed pass against
# k_weigh_stream, the batched tests (incl. the corrupt-descriptor report and the streaming packed batch), exact
# resample counts at C2-C5 sizes, the parity and frame-shape suites (deferred priors through every consumer);
# then an A/B of C4 / C5: default (pk + deferral), PFMPE_DIAG 16384 (no deferral), 4096|16384 (round-3 path);
# one SQ_INSTS_VALU pass of each weighing kernel at C4.  Logs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_weigh_pk.py tests/test_gpu_multi.py tests/test_gpu_resample_counts.py \
  tests/test_gpu_defer.py tests/test_gpu_bank_retable.py tests/test_gpu_grid_far.py tests/test_gpu_parity.py tests/test_gpu_frame_shapes.py -x -v \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04b_tests.log 2>&1; r=$?
grep -E "PASS|FAIL|ERROR|passed|failed|Error|assert" gpurun_out/r04b_tests.log | tail -40
[ $r -eq 0 ] || exit $r
for rep in 1 2; do
for c in C4 C5; do
  for d in 0 16384 20480; do
    timeout -k 10 300 python -u bench.py --config $c --steps 100 --warmup 10 --cpu-frames 0 --worst-frames 0 \
      --scale-ref-steps 0 --exact-steps 0 --multi-sweep none --diag $d > gpurun_out/r04b_bench_${c}_$d.log 2>&1 \
      || { tail -5 gpurun_out/r04b_bench_${c}_$d.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04b_bench_${c}_$d.log').read().strip().splitlines()[-1])
print('$c diag=$d', round(d['ms_per_step']*1e3,1), 'us/frame', round(d['value']/1e9,2), 'G/s', d['roofline'].get('per_kernel_avg_us'))"
  done
done
done
for d in 0 20480; do
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --output-format csv -d gpurun_out/r04b_pmc_$d -o run -- python3 bench.py --config C4 --steps 20 --warmup 3 \
    --cpu-frames 0 --no-timing --worst-frames 0 --scale-ref-steps 0 --exact-steps 0 --multi-sweep none --diag $d \
    > gpurun_out/r04b_pmc_$d.log 2>&1 || { tail -5 gpurun_out/r04b_pmc_$d.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for d in (0, 20480):
    f = glob.glob(f"gpurun_out/r04b_pmc_{d}/**/*counter_collection.csv", recursive=True)
    if not f: print("no csv", d); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for row in csv.DictReader(open(f[0])):
        k = row["Kernel_Name"].split("(")[0][-40:]
        acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
        n[(k, row["Counter_Name"])] += 1
    for k, c in acc.items():
        cnt = n[(k, "SQ_WAVES")] or 1
        w = c["SQ_WAVES"]
        print(d, k, "launches", cnt, "VALU/wave", round(c["SQ_INSTS_VALU"] / max(w, 1), 1), "SALU/wave",
              round(c["SQ_INSTS_SALU"] / max(w, 1), 1), "LDS/wave", round(c["SQ_INSTS_LDS"] / max(w, 1), 1),
              "waves/launch", w / cnt, "VALU per 64 particles", round(c["SQ_INSTS_VALU"] / cnt / (1e7 / 64), 1))
PY
# batched A/B: 32 x C5 (two concurrent batches) and 2 x C4 (one batch), default (packed batch pass + deferral) vs
# PFMPE_DIAG 16384 (no deferral: fp32 batches regenerate, fp16 batches materialise)
for d in 0 16384; do
  timeout -k 10 300 python -u bench.py --config C5 --steps 20 --warmup 5 --cpu-frames 0 --worst-frames 0 \
    --scale-ref-steps 0 --exact-steps 0 --multi-sweep 32 --multi-groups 2 --multi-steps 30 --diag $d \
    > gpurun_out/r04b_multi_C5_$d.log 2>&1 || { tail -5 gpurun_out/r04b_multi_C5_$d.log; exit 1; }
  timeout -k 10 300 python -u bench.py --config C4 --steps 20 --warmup 5 --cpu-frames 0 --worst-frames 0 \
    --scale-ref-steps 0 --exact-steps 0 --multi-sweep 2 --multi-groups 1 --multi-steps 30 --diag $d \
    > gpurun_out/r04b_multi_C4_$d.log 2>&1 || { tail -5 gpurun_out/r04b_multi_C4_$d.log; exit 1; }
  for c in C5 C4; do python3 -c "
import json; d=json.loads(open('gpurun_out/r04b_multi_${c}_$d.log').read().strip().splitlines()[-1])
print('$c diag=$d single', round(d['ms_per_step']*1e3,1), 'us', round(d['value']/1e9,2), 'G/s |',
      [(p['streams'], p['groups'], round(p['updates_per_s']/1e9,2), p['frac']) for p in d['multi_stream']['points']])"; done
done
