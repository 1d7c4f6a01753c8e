#!/bin/bash
# Unigram phase stamps (var/stamps) on both corpora, 64 MiB
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/uni_stamps; mkdir -p $O; export TMPDIR=/tmp
for c in fixture heldout; do
  SDL_LIB=var/stamps/libsdl_batcher.so timeout -k 10 150 python tools/uni_stamps.py 64 $c > $O/span_$c.txt 2>&1 || exit $?
done
grep -h -v amdgpu.ids $O/span_*.txt | grep -i "stamp\|uni\]" | head -80
