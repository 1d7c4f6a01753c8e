#!/bin/bash
# r03: GPU suite (all failures reported), smoke, rand-mode lines, Unigram A/B vs r02, WordPiece first-probe bound.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/suite; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1
echo "[pytest] exit $?" | tee -a $O/steps.log
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
bash tools/gpu_measure.sh "mlm_r1:--rng-mode 1 --no-cpu-baseline" "span_r1:--task span --rng-mode 1 --no-cpu-baseline" "span0:--task span --no-cpu-baseline" || exit $?
CORPORA=fixture TASK=span bash tools/gpu_ab.sh var/old/libsdl_batcher.so streaming_data_loader_amd/libsdl_batcher.so var/old/libsdl_batcher.so streaming_data_loader_amd/libsdl_batcher.so || exit $?
CORPORA="fixture heldout" TASK=mlm bash tools/gpu_ab.sh streaming_data_loader_amd/libsdl_batcher.so var/abl_fp/libsdl_batcher.so
