#!/bin/bash
# Where the WordPiece kernel's time goes on the fixture vs the held-out corpus:
# phase stamps and ablation builds (tools/build_variants.py stamps abl1 abl2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/hdiag; mkdir -p $O
export TMPDIR=/tmp
for c in fixture heldout; do
  SDL_LIB=build/var/stamps/libsdl_batcher.so timeout -k 10 120 python tools/wp_stamps.py ${TASK:-mlm} 64 $c > $O/stamps_$c.txt 2>&1 || exit $?
  for lib in streaming_data_loader_amd/libsdl_batcher.so build/var/abl1/libsdl_batcher.so build/var/abl2/libsdl_batcher.so; do
    SDL_LIB=$lib timeout -k 10 200 python bench.py --task ${TASK:-mlm} --steps 10 --warmup 2 --no-cpu-baseline --corpus $c > $O/b.json 2>>$O/b.err || exit $?
    python -c "import json;d=json.load(open('$O/b.json'));print('$c $lib', d['value'], d['stage_ms'])" | tee -a $O/ablate.txt
  done
done
