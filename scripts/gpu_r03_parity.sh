# Round 3: closed-loop tracker parity, the adversarial resampling boundary, the extended fp32 tolerance test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
PYT="python -u -m pytest -v -s --timeout 170 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PYT tests/test_gpu_closed_loop.py > gpurun_out/r03_closed_loop.log 2>&1; r1=$?
timeout -k 10 300 $PYT tests/test_gpu_resample_boundary.py > gpurun_out/r03_boundary.log 2>&1; r2=$?
timeout -k 10 400 $PYT tests/test_gpu_parity.py -k fp32_tolerance > gpurun_out/r03_fp32_tol.log 2>&1; r3=$?
tail -n 12 gpurun_out/r03_closed_loop.log gpurun_out/r03_boundary.log gpurun_out/r03_fp32_tol.log
echo "rc $r1 $r2 $r3"
exit $(( r1 | r2 | r3 ))
