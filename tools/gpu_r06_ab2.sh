#!/bin/bash
# r06: WordPiece A/B (mlm fixture + held-out kernel stats) of $BASELIB and the libraries given,
# then span kernel timelines (fixture, held-out) of the product library.  Output: gpurun_out/$OUT/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export OUT=${OUT:-r06ab2} TMPDIR=/tmp
for c in fixture heldout; do
  TASK=mlm CORPUS=$c BENCH_ARGS="--no-heldout" bash tools/gpu_prof.sh ${BASELIB:-var/base/libsdl_batcher.so} "$@" || exit $?
done
K=16 bash tools/gpu_trace.sh "--task span --no-heldout" "--task span --corpus heldout --no-heldout" || exit $?
