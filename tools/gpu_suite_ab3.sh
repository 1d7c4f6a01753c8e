#!/bin/bash
# Full GPU suite, then A/B (build/var/prev vs HEAD) on mlm, clm, span (fixture) and the gzip leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/suite.log 2>&1 || { tail -30 gpurun_out/ab/suite.log; exit 1; }
tail -1 gpurun_out/ab/suite.log
P=build/var/prev/libsdl_batcher.so; C=streaming_data_loader_amd/libsdl_batcher.so
for t in mlm clm span; do CORPORA=fixture TASK=$t tools/gpu_ab.sh $P $C $P $C || exit 1; done
tools/gpu_ab_gz.sh $P $C $P $C
for lib in $P $C $P $C; do
  SDL_LIB=$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --arena-mib 64 --no-cpu-baseline --json > gpurun_out/ab/j.json 2>> gpurun_out/ab/j.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab/j.json'))['provider_json']; print('json $lib', d['json_MBps'], d['ms'])"
done
