# The whole -m gpu suite + smoke, as the driver runs them at round end; logs under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_suite.log 2>&1; r=$?
tail -n 15 gpurun_out/gpu_suite.log
[ $r -eq 0 ] || exit $r
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; r=$?
tail -n 3 gpurun_out/smoke.log
exit $r
