#!/bin/bash
# r04: XCD-contiguous chunk mapping in k_wordpiece_chunks -- WordPiece parity, A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04u; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_size.py tests/test_gpu_testbin.py tests/test_gpu_drop_in.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1; rc=$?; tail -1 $O/test.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/test.log | head; exit $rc; }
CORPORA="fixture heldout" TASK=mlm bash tools/gpu_ab.sh var/xcd0/libsdl_batcher.so streaming_data_loader_amd/libsdl_batcher.so var/xcd0/libsdl_batcher.so streaming_data_loader_amd/libsdl_batcher.so
