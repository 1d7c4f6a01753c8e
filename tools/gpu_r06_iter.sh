#!/bin/bash
# r06 iteration: span/t5 GPU parity with $LIB (default: the product library), then rocprof
# kernel stats of span (fixture, then held-out) for $LIB and the variants given as arguments.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
LIB=${LIB:-streaming_data_loader_amd/libsdl_batcher.so}
SDL_LIB=$LIB OUT=${OUT:-r06iter}/tests bash tools/gpu_tests.sh ${TESTS:-tests/test_gpu_span.py tests/test_gpu_t5_kat.py} || exit $?
OUT=${OUT:-r06iter} BASELIB=$LIB bash tools/gpu_r06_prof.sh "$@"
