#!/bin/bash
# Times bench.py for several builds of libsdl_batcher.so, interleaved REPS times
# (A B C A B C ...).  Usage: tools/variants.sh lib1 lib2 ...   (BENCH_ARGS, REPS optional)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/variants.txt
for rep in $(seq ${REPS:-2}); do
  for lib in "$@"; do
    SDL_LIB=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/var.json 2>>gpurun_out/var.err
    rc=$?; [ $rc -ne 0 ] && { echo "$lib exit $rc"; exit $rc; }
    python -c "import json;d=json.load(open('gpurun_out/var.json'));s=d['stage_ms'];print('$lib', d['value'], s['tokenize'], s.get('rows'), s)" | tee -a gpurun_out/variants.txt
  done
done
