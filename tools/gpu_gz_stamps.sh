#!/bin/bash
# Inflate phase stamps (diagnostic SDL_STAMPS build) on the bench's BGZF stream.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/gz
SDL_LIB=var/stamps/libsdl_batcher.so timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --gz --no-cpu-baseline \
    --arena-mib 64 > gpurun_out/gz/stamps.json 2> gpurun_out/gz/stamps.err || { tail -20 gpurun_out/gz/stamps.err; exit 1; }
grep "gz stamps" gpurun_out/gz/stamps.err | tail -8
