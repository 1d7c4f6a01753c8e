#!/bin/bash
# WordPiece phase stamps (var/stamps) on the fixture and held-out corpora, 64 MiB.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/wps
for c in fixture heldout; do
  SDL_LIB=var/stamps/libsdl_batcher.so timeout -k 10 120 python tools/wp_stamps.py mlm 64 $c > gpurun_out/wps/$c.txt 2>&1 || exit $?
  echo "== $c"; grep -E "stamps" gpurun_out/wps/$c.txt
done
