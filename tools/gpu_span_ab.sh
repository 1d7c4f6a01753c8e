#!/bin/bash
# t5 parity tests, then A/B of build/var/prev against HEAD on span (fixture + held-out).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
timeout -k 10 500 python -u -m pytest tests/test_gpu_span.py tests/test_gpu_full_size.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/span_t.log 2>&1 || { tail -30 gpurun_out/ab/span_t.log; exit 1; }
tail -1 gpurun_out/ab/span_t.log
P=build/var/prev/libsdl_batcher.so; C=streaming_data_loader_amd/libsdl_batcher.so
CORPORA="fixture heldout" TASK=span tools/gpu_ab.sh $P $C $P $C
