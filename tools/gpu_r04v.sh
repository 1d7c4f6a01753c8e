#!/bin/bash
# r04: XCD-contiguous chunk map in all three chunk kernels -- full suite, A/B per task and corpus
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit $?
for t in mlm clm span; do
  CORPORA="fixture heldout" TASK=$t bash tools/gpu_ab.sh var/xcd0/libsdl_batcher.so streaming_data_loader_amd/libsdl_batcher.so || exit $?
done
