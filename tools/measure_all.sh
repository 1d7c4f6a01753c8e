#!/bin/bash
# One GPU-box session producing every number DESIGN.md quotes:
#   GPU parity suite, smoke, the default bench (mlm, with CPU baseline), the
#   other BASELINE configs, end-to-end host-path rates, a rocprofv3 kernel-trace
#   summary per task and the PMC passes of the mlm tokenize kernel.
# Each GPU step has its own time limit; a fault/abort/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/final
mkdir -p $O
export TMPDIR=/tmp
step() {  # step NAME LIMIT CMD...: stop on anything but success
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  echo "[$name] exit $rc" >> $O/steps.log; echo "[$name] exit $rc" >&2
  [ $rc -eq 0 ] || exit $rc
}
STEPS="${1:-tests,bench,tasks,e2e,prof,pmc}"
[[ $STEPS == *tests* ]] && step pytest 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf -o log_cli=false > $O/pytest_gpu.log 2>&1
[[ $STEPS == *tests* ]] && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
[[ $STEPS == *bench* ]] && step bench 600 python bench.py > $O/bench_mlm.json 2> $O/bench_mlm.err
if [[ $STEPS == *tasks* ]]; then
  for t in span clm multi-label single-class; do
    step bench_$t 600 python bench.py --task $t --frames > $O/bench_$t.json 2> $O/bench_$t.err
  done
  step bench_mlm_frames 300 python bench.py --frames --e2e-frames --no-cpu-baseline > $O/bench_mlm_frames.json 2> $O/bench_mlm_frames.err
fi
[[ $STEPS == *json* ]] && step bench_json 300 python bench.py --steps 5 --warmup 2 --arena-mib 64 --no-cpu-baseline --json > $O/bench_json.json 2> $O/bench_json.err
if [[ $STEPS == *e2e* ]]; then
  for t in mlm span clm multi-label single-class; do
    step e2e_$t 300 python bench.py --task $t --steps 3 --warmup 1 --arena-mib 64 --no-cpu-baseline --e2e > $O/e2e_$t.json 2> $O/e2e_$t.err
  done
fi
if [[ $STEPS == *prof* ]]; then
  for t in mlm span clm multi-label single-class; do
    step prof_$t 300 rocprofv3 --kernel-trace --stats -d $O/prof_$t -o run --output-format csv -- python3 bench.py --task $t --steps 5 --warmup 2 --no-cpu-baseline --frames > $O/prof_$t.json 2> $O/prof_$t.err
  done
fi
if [[ $STEPS == *pmc* ]]; then
  PMC_BENCH_ARGS="--steps 2 --warmup 1 --arena-mib 256 --no-cpu-baseline --frames" step pmc 900 tools/pmc.sh
fi
echo all done | tee -a $O/steps.log
