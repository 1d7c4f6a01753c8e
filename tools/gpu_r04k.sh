#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04k; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gpt2.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread -k "gpt2 or clm" > $O/test.log 2>&1; rc=$?; tail -1 $O/test.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/test.log | head; exit $rc; }
CORPORA="heldout fixture" TASK=clm bash tools/gpu_ab.sh var/bl1024/libsdl_batcher.so var/bl4096/libsdl_batcher.so streaming_data_loader_amd/libsdl_batcher.so
