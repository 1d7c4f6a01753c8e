#!/bin/bash
# r04: k_rows writes a small mlm / clm push's rows into the host batches -- suite, push latency, big-path A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04t; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit $?
PUSH_TAG=7 bash tools/gpu_push.sh || exit $?
bash tools/gpu_push_c.sh || exit $?
for t in mlm clm; do
  for lib in var/head2/libsdl_batcher.so streaming_data_loader_amd/libsdl_batcher.so; do
    SDL_LIB=$lib timeout -k 10 200 python bench.py --task $t --steps 10 --warmup 2 --no-cpu-baseline > $O/b.json 2>>$O/b.err || exit $?
    python -c "import json;d=json.load(open('$O/b.json'));print('$t $lib', d['value'], 'rows', d['stage_ms']['rows'])" | tee -a $O/ab.txt
  done
done
