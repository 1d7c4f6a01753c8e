#!/bin/bash
# r06 Unigram A/B: rocprof kernel stats (fixture + held-out) of span for the product library and
# variants given as arguments (var/NAME/libsdl_batcher.so).  Output: gpurun_out/${OUT:-r06prof}/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export OUT=${OUT:-r06prof} TASK=${TASK:-span}
O=gpurun_out/$OUT; mkdir -p $O
for c in ${CORPORA:-fixture heldout}; do
  CORPUS=$c BENCH_ARGS="--no-heldout" bash tools/gpu_prof.sh ${BASELIB:-streaming_data_loader_amd/libsdl_batcher.so} "$@" || exit $?
done
