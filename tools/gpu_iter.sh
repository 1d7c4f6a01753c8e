#!/bin/bash
# One GPU iteration: the GPU parity suite, then tokenize-stage timings of the
# product library against variant builds (tools/variants.sh) for the tasks given.
#   tools/gpu_iter.sh "span mlm" build/v_old/libsdl_batcher.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
tasks=$1; shift
: > gpurun_out/iter.txt
for t in $tasks; do
  BENCH_ARGS="--task $t" bash tools/variants.sh streaming_data_loader_amd/libsdl_batcher.so "$@" || exit $?
  sed "s/^/$t /" gpurun_out/variants.txt >> gpurun_out/iter.txt
done
cat gpurun_out/iter.txt
