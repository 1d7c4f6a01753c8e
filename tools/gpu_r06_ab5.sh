#!/bin/bash
# r06: full GPU suite + smoke of the product, span kernel stats (fixture, held-out) of the product
# and the variants given, and the held-out span timeline.  Output: gpurun_out/${OUT:-r06ab5}/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export OUT=${OUT:-r06ab5} TMPDIR=/tmp
bash tools/gpu_suite.sh || exit $?
for c in fixture heldout; do
  TASK=span CORPUS=$c BENCH_ARGS="--no-heldout" bash tools/gpu_prof.sh streaming_data_loader_amd/libsdl_batcher.so "$@" || exit $?
done
K=40 bash tools/gpu_trace.sh "--task span --corpus heldout --no-heldout" || exit $?
