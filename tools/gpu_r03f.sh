#!/bin/bash
# r03: full GPU suite + smoke, then span A/B (r02 lib vs HEAD) on both corpora.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/suite; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1
echo "[pytest] exit $?" | tee -a $O/steps.log; tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
CORPORA="fixture heldout" TASK=span bash tools/gpu_ab.sh var/old/libsdl_batcher.so streaming_data_loader_amd/libsdl_batcher.so
