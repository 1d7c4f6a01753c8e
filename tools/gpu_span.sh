set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_span.py -x -v --timeout 300 --timeout-method thread > gpurun_out/span.log 2>&1
rc=$?
tail -40 gpurun_out/span.log
exit $rc
