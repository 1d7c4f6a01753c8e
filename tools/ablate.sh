#!/bin/bash
# Times the full tokenize kernel against diagnostic builds with phases removed.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in streaming_data_loader_amd/libsdl_batcher.so build/abl1/libsdl_batcher.so build/abl2/libsdl_batcher.so build/abl3/libsdl_batcher.so; do
  SDL_LIB=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/abl.json 2>>gpurun_out/abl.err
  rc=$?; [ $rc -ne 0 ] && { echo "$lib exit $rc"; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/abl.json'));print('$lib', d['stage_ms'])" | tee -a gpurun_out/ablate.txt
done
