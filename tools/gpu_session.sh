#!/bin/bash
# One GPU-box session: STEPS (comma list) of
#   tests   GPU parity suite + smoke
#   bench   bench.py default (mlm) + span + clm (+ held-out corpus)
#   e2e     end-to-end host paths (incl. channel per-record vs drained)
#   prof    rocprofv3 --kernel-trace --stats per task
#   pmc     PMC passes per task (tools/pmc.sh) -> gpurun_out/pmc_*
# Output under gpurun_out/$TAG.  Each GPU step has its own time limit; a
# fault/abort/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG="${TAG:-s}"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
step() {  # step NAME LIMIT CMD...: stop on anything but success
  local name=$1 lim=$2; shift 2
  local t0=$(date +%s)
  timeout -k 10 "$lim" "$@"
  local rc=$?
  echo "[$name] exit $rc ($(( $(date +%s) - t0 )) s)" | tee -a $O/steps.log >&2
  [ $rc -eq 0 ] || exit $rc
}
STEPS="${1:-tests,bench}"
TASKS="${TASKS:-mlm span clm}"
if [[ $STEPS == *tests* ]]; then
  step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -rf ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
fi
if [[ $STEPS == *bench* ]]; then
  for t in $TASKS; do
    step bench_$t 400 python bench.py --task $t > $O/bench_$t.json 2> $O/bench_$t.err
  done
fi
if [[ $STEPS == *heldout* ]]; then
  for t in $TASKS; do
    step heldout_$t 300 python bench.py --task $t --corpus heldout --no-cpu-baseline > $O/heldout_$t.json 2> $O/heldout_$t.err
  done
fi
if [[ $STEPS == *e2e* ]]; then
  for t in $TASKS; do
    step e2e_$t 300 python bench.py --task $t --steps 3 --warmup 1 --arena-mib 64 --no-cpu-baseline --e2e > $O/e2e_$t.json 2> $O/e2e_$t.err
  done
fi
if [[ $STEPS == *prof* ]]; then
  for t in $TASKS; do
    step prof_$t 300 rocprofv3 --kernel-trace --stats -d $O/prof_$t -o run --output-format csv -- python3 bench.py --task $t --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_$t.json 2> $O/prof_$t.err
  done
fi
if [[ $STEPS == *pmc* ]]; then
  for t in $TASKS; do
    step pmc_$t 1000 tools/pmc.sh $t 256
  done
fi
echo all done | tee -a $O/steps.log
