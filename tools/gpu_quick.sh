#!/bin/bash
# GPU tests selected by -k "$K" (all GPU tests when K is empty), then
# tools/gpu_measure.sh with the arguments.  e.g.
#   K="span" bash tools/gpu_quick.sh "span:--task span --no-cpu-baseline"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/suite; rm -rf $O gpurun_out/meas gpurun_out/ab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu ${K:+-k "$K"} -v --timeout 120 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1
rc=$?; echo "[pytest] exit $rc" | tee -a $O/steps.log; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
[ $# -eq 0 ] || bash tools/gpu_measure.sh "$@"
