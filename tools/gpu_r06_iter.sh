#!/bin/bash
# r06 iteration: span/t5 GPU parity with the product library, then rocprof kernel stats of span
# (fixture, then held-out) for the product library and the variants given as arguments.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-r06iter}/tests bash tools/gpu_tests.sh ${TESTS:-tests/test_gpu_span.py tests/test_gpu_t5_kat.py} || exit $?
OUT=${OUT:-r06iter} bash tools/gpu_r06_prof.sh "$@"
