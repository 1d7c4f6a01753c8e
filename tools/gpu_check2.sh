#!/bin/bash
# Full GPU suite + single-class bench (+frames, e2e) + frames for multi-label.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/check2
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  echo "[$name] exit $rc" >> $O/steps.log; echo "[$name] exit $rc" >&2
  [ $rc -eq 0 ] || exit $rc
}
step pytest 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -rf > $O/pytest.log 2>&1
step bench_sc 400 python bench.py --task single-class --frames > $O/bench_single-class.json 2> $O/bench_single-class.err
step e2e_sc 300 python bench.py --task single-class --steps 3 --warmup 1 --arena-mib 64 --no-cpu-baseline --e2e > $O/e2e_single-class.json 2> $O/e2e_single-class.err
step prof_sc 300 rocprofv3 --kernel-trace --stats -d $O/prof_sc -o run --output-format csv -- python3 bench.py --task single-class --steps 5 --warmup 2 --frames --no-cpu-baseline > $O/prof_sc.json 2> $O/prof_sc.err
echo all done | tee -a $O/steps.log
