#!/bin/bash
# bench lines (fixture, every task; PMC traffic from profiles/pmc) + rocprof kernel stats.
# PART=a: mlm clm span multi-label single-class with CPU baselines and rocprof; PART=b: held-out
# and rng_mode 1 lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-final}; mkdir -p $O; export TMPDIR=/tmp
if [ "${PART:-a}" = a ]; then
  for t in ${TASKS:-mlm clm span multi-label single-class}; do
    timeout -k 10 240 python bench.py --task $t > $O/bench_$t.json 2> $O/bench_$t.err || exit $?
    tail -c 300 $O/bench_$t.json; echo
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$t -o run -- python3 bench.py --task $t --no-cpu-baseline > $O/prof_$t.out 2>&1 || exit $?
    find $O/prof_$t -name '*kernel_trace.csv' -delete  # (the per-dispatch trace: > 64 MiB over the tasks; the stats stay)
  done
else
  for t in mlm clm span; do
    timeout -k 10 240 python bench.py --task $t --corpus heldout --no-cpu-baseline > $O/heldout_$t.json 2> $O/heldout_$t.err || exit $?
  done
  for t in mlm span; do
    timeout -k 10 240 python bench.py --task $t --rng-mode 1 --no-cpu-baseline > $O/rng1_$t.json 2> $O/rng1_$t.err || exit $?
  done
  ls $O
fi
