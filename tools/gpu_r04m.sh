#!/bin/bash
# r04: span rows in two phases -- parity (span tests), then A/B vs the one-pass kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04m; mkdir -p $O; export TMPDIR=/tmp
SDL_SPAN_TWO_PHASE=1 SDL_SMALL_CALLS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_span.py tests/test_gpu_push_direct.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1; rc=$?; tail -1 $O/test.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/test.log | head -20; exit $rc; }
for rm in 0 1; do
  for one in 1 0; do
    SDL_SPAN_TWO_PHASE=$((1-one)) SDL_SMALL_CALLS=1 timeout -k 10 200 python bench.py --task span --steps 10 --warmup 2 --no-cpu-baseline --rng-mode $rm > $O/b.json 2>>$O/b.err || exit $?
    python -c "import json;d=json.load(open('$O/b.json'));print('span rng$rm onepass=$one', d['value'], d['stage_ms'])" | tee -a $O/ab.txt
  done
done
SDL_SPAN_TWO_PHASE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --task span --steps 10 --warmup 2 --no-cpu-baseline > $O/prof.out 2>&1 || exit $?
