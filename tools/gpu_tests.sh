#!/bin/bash
# Selected GPU test files (arguments), then optional extra commands in $AFTER.
#   bash tools/gpu_tests.sh tests/test_gpu_span.py tests/test_gpu_t5_kat.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-tests}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 ${LIMIT:-600} python -u -m pytest "$@" -m gpu -x -v --timeout 120 --timeout-method thread -rf > $O/pytest.log 2>&1
rc=$?; echo "[pytest] exit $rc"; grep -E "passed|failed|FAILED|Error" $O/pytest.log | tail -15; [ $rc -eq 0 ] || exit $rc
if [ -n "${AFTER:-}" ]; then bash -c "$AFTER" || exit $?; fi
