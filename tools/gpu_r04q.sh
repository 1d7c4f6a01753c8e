#!/bin/bash
# r04: per-record pushes without the k_chunk_ranges launch -- suite, push latency, A/B of the big path
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04q; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit $?
PUSH_TAG=5 bash tools/gpu_push.sh || exit $?
for t in mlm clm span; do
  for lib in var/pre_prefetch/libsdl_batcher.so streaming_data_loader_amd/libsdl_batcher.so; do
    SDL_LIB=$lib timeout -k 10 200 python bench.py --task $t --steps 10 --warmup 2 --no-cpu-baseline > $O/b.json 2>>$O/b.err || exit $?
    python -c "import json;d=json.load(open('$O/b.json'));print('$t $lib', d['value'], d['stage_ms'])" | tee -a $O/ab.txt
  done
done
