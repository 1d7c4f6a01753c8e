#!/bin/bash
# rocprofv3 kernel statistics of bench.py on the held-out corpus, per task.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/hprof; mkdir -p $O
export TMPDIR=/tmp
for t in ${TASKS:-clm span}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$t -o run --output-format csv -- python3 bench.py --task $t --steps 5 --warmup 2 --no-cpu-baseline --corpus ${CORPUS:-heldout} > $O/$t.json 2> $O/$t.err || exit $?
done
