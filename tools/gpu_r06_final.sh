#!/bin/bash
# r06 final: GPU suite + smoke, every task's bench line + rocprof kernel stats (fixture), held-out
# and rng_mode 1 lines, per-record push latency.  Output: gpurun_out/r06final/, gpurun_out/push_r06/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit $?
OUT=r06final bash tools/gpu_final.sh || exit $?
OUT=r06final PART=b bash tools/gpu_final.sh || exit $?
PUSH_TAG=_r06 bash tools/gpu_push.sh || exit $?
find gpurun_out/push_r06 -name '*kernel_trace.csv' -delete
