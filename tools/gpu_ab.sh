#!/bin/bash
# A/B: bench stage times of several libsdl_batcher.so builds on the fixture
# and held-out corpora.  Usage: TASK=mlm tools/gpu_ab.sh lib1 lib2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab; mkdir -p $O
export TMPDIR=/tmp
for c in ${CORPORA:-fixture heldout}; do
  for lib in "$@"; do
    SDL_LIB=$lib timeout -k 10 200 python bench.py --task ${TASK:-mlm} --steps 10 --warmup 2 --no-cpu-baseline --corpus $c ${BENCH_ARGS:-} > $O/b.json 2>>$O/b.err || exit $?
    python -c "import json;d=json.load(open('$O/b.json'));print('$c $lib', d['value'], d['stage_ms'])" | tee -a $O/ab.txt
  done
done
