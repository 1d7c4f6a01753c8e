#!/bin/bash
# Phase-stamp splits (var/stamps, diagnostic build) of the three chunk kernels
# on both corpora, 64 MiB arena: gpurun_out/stamps/<task>_<corpus>.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/stamps; mkdir -p $O
export TMPDIR=/tmp
for c in fixture heldout; do
  SDL_LIB=var/stamps/libsdl_batcher.so timeout -k 10 150 python tools/uni_stamps.py 64 $c > $O/span_$c.txt 2>&1 || exit $?
  for t in mlm clm; do
    SDL_LIB=var/stamps/libsdl_batcher.so timeout -k 10 150 python tools/wp_stamps.py $t 64 $c > $O/${t}_$c.txt 2>&1 || exit $?
  done
done
grep -h -v amdgpu.ids $O/*.txt | grep -i "stamp" | head -80
