#!/bin/bash
# r06: GPU parity of every tokenizer with $PARITY_LIB, then mlm / clm / span kernel stats
# (fixture, held-out) of the product and the variants given.  Output: gpurun_out/${OUT:-r06ab11}/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export OUT=${OUT:-r06ab11} TMPDIR=/tmp
O=gpurun_out/$OUT; mkdir -p $O
SDL_LIB=$PARITY_LIB timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gpt2.py tests/test_gpu_span.py tests/test_gpu_t5_kat.py tests/test_gpu_testbin.py tests/test_gpu_wordpiece_groups.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for t in mlm clm span; do
  for c in fixture heldout; do
    TASK=$t CORPUS=$c BENCH_ARGS="--no-heldout" bash tools/gpu_prof.sh streaming_data_loader_amd/libsdl_batcher.so "$@" || exit $?
  done
done
