#!/bin/bash
# Transport frames on the GPU: parity tests, bench --frames per task, rocprof stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/frames
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  echo "[$name] exit $rc" >> $O/steps.log; echo "[$name] exit $rc" >&2
  [ $rc -eq 0 ] || exit $rc
}
step pytest 300 python -u -m pytest tests/test_pickle_frames.py tests/test_abi.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for t in ${TASKS:-mlm clm span multi-label}; do
  step bench_$t 300 python bench.py --task $t --steps 10 --warmup 2 --frames --no-cpu-baseline > $O/bench_$t.json 2> $O/bench_$t.err
done
[[ ${CPU:-1} == 1 ]] && step bench_mlm_cpu 300 python bench.py --task mlm --steps 5 --warmup 2 --frames > $O/bench_mlm_cpu.json 2> $O/bench_mlm_cpu.err
step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --task mlm --steps 5 --warmup 2 --frames --no-cpu-baseline > $O/prof.json 2> $O/prof.err
echo all done | tee -a $O/steps.log
