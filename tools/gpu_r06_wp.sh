#!/bin/bash
# r06 WordPiece iteration: GPU suite + smoke, then rocprof kernel stats of mlm (fixture and
# held-out) for $BASELIB and the product library, then the default bench line.
# Output: gpurun_out/${OUT:-r06wp}/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export OUT=${OUT:-r06wp} TMPDIR=/tmp
O=gpurun_out/$OUT; mkdir -p $O
if [ -z "${NO_SUITE:-}" ]; then bash tools/gpu_suite.sh || exit $?; fi
for c in fixture heldout; do
  TASK=${TASK:-mlm} CORPUS=$c BENCH_ARGS="--no-heldout" bash tools/gpu_prof.sh ${BASELIB:-var/base/libsdl_batcher.so} streaming_data_loader_amd/libsdl_batcher.so || exit $?
done
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
tail -c 600 $O/bench_default.json
