#!/bin/bash
# r04: k_bpe_long from a shared cursor, 2048 waves -- clm parity, A/B on both corpora
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04r; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gpt2.py tests/test_gpu_full_size.py tests/test_gpu_push_direct.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1; rc=$?; tail -1 $O/test.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/test.log | head; exit $rc; }
CORPORA="fixture heldout" TASK=clm bash tools/gpu_ab.sh var/head_r04/libsdl_batcher.so streaming_data_loader_amd/libsdl_batcher.so
