#!/bin/bash
# Phase split of the t5 chunk kernel (diagnostic stamps build, 256 MiB bench arena).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SDL_LIB=var/stamps/libsdl_batcher.so timeout -k 10 120 python tools/uni_stamps.py 256 > gpurun_out/stamps.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/stamps.txt; exit $rc
