#!/bin/bash
# r03: inflate fuzz GPU tests; Unigram A/B r02 lib / HEAD / HEAD with the r02 Unigram source.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03e; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_inflate_fuzz.py tests/test_inflate.py -m gpu -v --timeout 120 --timeout-method thread -rf > $O/pytest.log 2>&1
echo "[pytest] exit $?" | tee -a $O/steps.log; tail -1 $O/pytest.log
CORPORA=fixture TASK=span bash tools/gpu_ab.sh var/old/libsdl_batcher.so streaming_data_loader_amd/libsdl_batcher.so var/uni_r02/libsdl_batcher.so var/old/libsdl_batcher.so streaming_data_loader_amd/libsdl_batcher.so var/uni_r02/libsdl_batcher.so
