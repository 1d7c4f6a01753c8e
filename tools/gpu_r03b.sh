#!/bin/bash
# r03: GPU suite, then the rand-mode mlm line and the Unigram A/B against the r02 library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_suite.sh || exit $?
bash tools/gpu_measure.sh "mlm_r1:--rng-mode 1 --no-cpu-baseline" "span_r1:--task span --rng-mode 1 --no-cpu-baseline" || exit $?
CORPORA=fixture TASK=span bash tools/gpu_ab.sh var/old/libsdl_batcher.so streaming_data_loader_amd/libsdl_batcher.so var/old/libsdl_batcher.so streaming_data_loader_amd/libsdl_batcher.so
