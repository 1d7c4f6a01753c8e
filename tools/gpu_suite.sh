#!/bin/bash
# GPU parity suite + smoke on the box.  Output: gpurun_out/suite/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/suite; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
step() {  # step NAME LIMIT CMD...: stop on anything but success
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  echo "[$name] exit $rc" >> $O/steps.log; echo "[$name] exit $rc" >&2
  [ $rc -eq 0 ] || exit $rc
}
step pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -rf ${SUITE_K:+-k "$SUITE_K"} > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
