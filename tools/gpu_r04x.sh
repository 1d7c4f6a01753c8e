#!/bin/bash
# r04: WordPiece waves per EU 4 / 5 (default) / 6 with the XCD chunk map
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CORPORA="fixture heldout" TASK=mlm bash tools/gpu_ab.sh streaming_data_loader_amd/libsdl_batcher.so var/wp6/libsdl_batcher.so var/wp4/libsdl_batcher.so streaming_data_loader_amd/libsdl_batcher.so var/wp6/libsdl_batcher.so
