#!/bin/bash
# GPU parity suite, then A/B (prev vs current lib) and instruction mix for one task.
# Usage: TASK=span tools/gpu_abt.sh   (prev lib: build/var/prev/libsdl_batcher.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -rf gpurun_out/ab
P=build/var/prev/libsdl_batcher.so
C=streaming_data_loader_amd/libsdl_batcher.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
tools/gpu_ab.sh $P $C $P $C || exit 1
tools/gpu_insts.sh $P $C
