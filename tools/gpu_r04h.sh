#!/bin/bash
# fused rand set check + Unigram ablation timings
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04h; mkdir -p $O; export TMPDIR=/tmp
OUT=r04h bash tools/gpu_r04b.sh || exit $?
CORPORA="fixture heldout" TASK=span bash tools/gpu_ab.sh streaming_data_loader_amd/libsdl_batcher.so var/uabl1/libsdl_batcher.so var/uabl2/libsdl_batcher.so
