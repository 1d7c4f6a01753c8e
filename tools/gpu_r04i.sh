#!/bin/bash
# Unigram DP lane-per-job variant: parity (t5 tests on the variant), then A/B span timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04i; mkdir -p $O; export TMPDIR=/tmp
V=${V:-var/dpg1/libsdl_batcher.so}
SDL_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_span.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread -k "span or t5" > $O/test.log 2>&1; rc=$?; tail -1 $O/test.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/test.log | head; exit $rc; }
CORPORA="fixture heldout" TASK=span bash tools/gpu_ab.sh streaming_data_loader_amd/libsdl_batcher.so $V
