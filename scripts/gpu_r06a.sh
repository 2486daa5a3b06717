#!/bin/bash
# Round 6 (a): C3 parity + the driver's bench command and its kernel trace on the round's start tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -s -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_packed_oracle.py "tests/test_gpu_frame_shapes.py::test_streaming_weighing_is_bit_identical" \
  tests/test_gpu_closed_loop.py > gpurun_out/r06/parity_c3.txt 2>&1 || { tail -40 gpurun_out/r06/parity_c3.txt; exit 1; }
tail -n 3 gpurun_out/r06/parity_c3.txt
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/bench_driver_a.log 2>&1 || { tail -20 gpurun_out/r06/bench_driver_a.log; exit 1; }
tail -c 3000 gpurun_out/r06/bench_driver_a.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/trace_a -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/trace_a.log 2>&1 || { tail -20 gpurun_out/r06/trace_a.log; exit 1; }
echo trace done
