#!/bin/bash
# bench.py for one task + a rocprofv3 kernel-trace of the same command.
# usage: tools/gpu_bench_task.sh TASK [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=$1; shift
timeout -k 10 600 python bench.py --task $T --steps 10 --warmup 3 "$@" > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; echo "[bench $T] exit $rc"; cat gpurun_out/bench_$T.json; tail -4 gpurun_out/bench_$T.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python3 bench.py --task $T --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$T.json 2> gpurun_out/prof_$T.err
rc=$?; echo "[rocprof $T] exit $rc"
find gpurun_out/prof_$T -name '*kernel_stats*' -exec head -12 {} \;
exit $rc
