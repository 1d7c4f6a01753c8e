#!/bin/bash
# Full GPU suite, then A/B of the committed-tree library (build/var/prev) against HEAD for TASK (default mlm).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/suite.log 2>&1 || { tail -30 gpurun_out/ab/suite.log; exit 1; }
tail -1 gpurun_out/ab/suite.log
P=build/var/prev/libsdl_batcher.so; C=streaming_data_loader_amd/libsdl_batcher.so
CORPORA=${CORPORA:-fixture heldout} TASK=${TASK:-mlm} tools/gpu_ab.sh $P $C $P $C
