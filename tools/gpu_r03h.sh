#!/bin/bash
# r03: Unigram tests, then span A/B (var/head vs HEAD) on both corpora.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/suite; rm -rf $O gpurun_out/ab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -k "${K:-span or heldout or t5 or unigram or full_size}" -v --timeout 120 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1
rc=$?; echo "[pytest] exit $rc" | tee -a $O/steps.log; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
CORPORA="fixture heldout" TASK=span bash tools/gpu_ab.sh var/head/libsdl_batcher.so streaming_data_loader_amd/libsdl_batcher.so
