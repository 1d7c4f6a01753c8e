#!/bin/bash
# Pipelined-segment check: GPU tests of the touched paths, then the mlm bench at
# several segment counts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-seg}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.log 2>&1 || { echo "pytest rc $?"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for K in ${SEGS:-1 2 4 8}; do
  SDL_SEGMENTS=$K timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench_k$K.json 2> $O/bench_k$K.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_k$K.json'));print('K=$K', d['value'], d['ms_per_step'], d['stage_ms'])"
done
