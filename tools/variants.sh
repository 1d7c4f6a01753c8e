#!/bin/bash
# Times the tokenize stage of bench.py for several builds of libsdl_batcher.so
# (product lib first).  Usage: tools/variants.sh lib1 lib2 ...   (BENCH_ARGS optional)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/variants.txt
for lib in "$@"; do
  SDL_LIB=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/var.json 2>>gpurun_out/var.err
  rc=$?; [ $rc -ne 0 ] && { echo "$lib exit $rc"; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/var.json'));print('$lib', d['value'], d['stage_ms'])" | tee -a gpurun_out/variants.txt
done
