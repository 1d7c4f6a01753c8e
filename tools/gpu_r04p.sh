#!/bin/bash
# r04: row prefetch (k_rows, k_span_write) -- parity, then A/B against the build before it
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04p; mkdir -p $O; export TMPDIR=/tmp
SDL_SMALL_CALLS=1 SDL_SPAN_TWO_PHASE=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1; rc=$?; tail -1 $O/test.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/test.log | head -20; exit $rc; }
for t in mlm clm multi-label span; do
  for lib in var/pre_prefetch/libsdl_batcher.so streaming_data_loader_amd/libsdl_batcher.so; do
    for tp in 0 1; do
      [ $t != span ] && [ $tp = 1 ] && continue
      SDL_SPAN_TWO_PHASE=$tp SDL_LIB=$lib timeout -k 10 200 python bench.py --task $t --steps 10 --warmup 2 --no-cpu-baseline > $O/b.json 2>>$O/b.err || exit $?
      python -c "import json;d=json.load(open('$O/b.json'));print('$t $lib tp=$tp', d['value'], 'rows', d['stage_ms']['rows'])" | tee -a $O/ab.txt
    done
  done
done
