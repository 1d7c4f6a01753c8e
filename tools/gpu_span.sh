#!/bin/bash
# GPU session for the t5/span path: its parity tests first, then the whole GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_span.py -x -v --timeout 300 --timeout-method thread > gpurun_out/span.log 2>&1
rc=$?
tail -40 gpurun_out/span.log
case $rc in 0|1) ;; *) echo "stopping: span tests exit $rc"; exit $rc;; esac
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1
rc2=$?
tail -15 gpurun_out/pytest_gpu.log
exit $(( rc > rc2 ? rc : rc2 ))
