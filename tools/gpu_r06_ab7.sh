#!/bin/bash
# r06: span/t5 GPU parity with $PARITY_LIB, then span kernel stats (fixture, held-out) of the
# product and the variants given.  Output: gpurun_out/${OUT:-r06ab7}/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export OUT=${OUT:-r06ab7} TMPDIR=/tmp
O=gpurun_out/$OUT; mkdir -p $O
SDL_LIB=$PARITY_LIB timeout -k 10 600 python -u -m pytest tests/test_gpu_span.py tests/test_gpu_t5_kat.py tests/test_gpu_push_direct.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in fixture heldout; do
  TASK=span CORPUS=$c BENCH_ARGS="--no-heldout" bash tools/gpu_prof.sh streaming_data_loader_amd/libsdl_batcher.so "$@" || exit $?
done
