#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/dbg; mkdir -p $O; export TMPDIR=/tmp SDL_SPAN_TWO_PHASE=1
for lib in streaming_data_loader_amd/libsdl_batcher.so var/sp_tab0/libsdl_batcher.so var/sp_mk16/libsdl_batcher.so; do
  echo "== $lib"
  SDL_LIB=$lib timeout -k 10 120 python tools/debug_span.py 128 8 16.0 2.0 0 2>&1 | grep -v amdgpu.ids | tail -4 || exit $?
done
