#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
C=streaming_data_loader_amd/libsdl_batcher.so
CORPORA="fixture heldout" TASK=mlm tools/gpu_ab.sh $C build/var/rare/libsdl_batcher.so $C build/var/rare/libsdl_batcher.so
