#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Each GPU step has its own time limit; a fault/abort/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() {  # test failures (1) continue; faults, aborts, timeouts stop
  local rc=$1 step=$2
  echo "[$step] exit $rc" | tee -a gpurun_out/steps.log
  case $rc in 0|1) return 0;; *) echo "stopping after $step" | tee -a gpurun_out/steps.log; exit $rc;; esac
}
STEPS="${1:-tests,smoke,bench,prof}"
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 600 -rf > gpurun_out/pytest_gpu.log 2>&1
  stop_on_fault $? pytest
  tail -30 gpurun_out/pytest_gpu.log
fi
if [[ $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  stop_on_fault $? smoke
  tail -3 gpurun_out/smoke.log
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 600 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  stop_on_fault $? bench
  cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
fi
if [[ $STEPS == *e2e* ]]; then
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --arena-mib 64 --no-cpu-baseline --e2e > gpurun_out/bench_e2e.json 2> gpurun_out/bench_e2e.err
  stop_on_fault $? e2e
  cat gpurun_out/bench_e2e.json
fi
if [[ $STEPS == *prof* ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
  stop_on_fault $? rocprof
  find gpurun_out/prof -name '*stats*' | head
fi
