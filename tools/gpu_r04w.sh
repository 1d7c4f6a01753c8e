#!/bin/bash
# r04: Unigram long items from a shared cursor -- span parity, A/B both corpora
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04w; mkdir -p $O; export TMPDIR=/tmp
SDL_LIB=var/uni_cursor/libsdl_batcher.so timeout -k 10 600 python -u -m pytest tests/test_gpu_span.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1; rc=$?; tail -1 $O/test.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/test.log | head; exit $rc; }
CORPORA="fixture heldout" TASK=span bash tools/gpu_ab.sh var/head3/libsdl_batcher.so var/uni_cursor/libsdl_batcher.so var/head3/libsdl_batcher.so var/uni_cursor/libsdl_batcher.so
