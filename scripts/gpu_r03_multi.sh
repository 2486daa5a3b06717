# Round 3: the batched path after the bounds audit / hardening, smallest first; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 170 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PYT tests/test_gpu_multi.py -k "equals_single or fp64_stream or rejects or block_limit or interleaved" > gpurun_out/r03_multi_small.log 2>&1 &&
timeout -k 10 200 $PYT tests/test_gpu_multi.py -k "large_fp16_streams_bit_identical and 3000000" > gpurun_out/r03_multi_3M.log 2>&1 &&
timeout -k 10 240 $PYT tests/test_gpu_multi.py -k "large_fp16_streams_bit_identical and 10000000" > gpurun_out/r03_multi_10M.log 2>&1 &&
timeout -k 10 300 $PYT tests/test_gpu_multi.py -k "large_concurrent" > gpurun_out/r03_multi_conc.log 2>&1
rc=$?
tail -n 4 gpurun_out/r03_multi_*.log
exit $rc
