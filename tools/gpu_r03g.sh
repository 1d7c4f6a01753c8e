#!/bin/bash
# r03: rand-mode GPU parity, mlm rng1 timing + kernel stats, span word-table A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/suite; rm -rf $O gpurun_out/meas gpurun_out/ab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -k "rand or span or mlm" -v --timeout 120 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1
rc=$?; echo "[pytest] exit $rc" | tee -a $O/steps.log; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_measure.sh "mlm_r1:--rng-mode 1 --no-cpu-baseline" "prof/mlm_r1:--rng-mode 1 --no-cpu-baseline" || exit $?
CORPORA="fixture heldout" TASK=span bash tools/gpu_ab.sh streaming_data_loader_amd/libsdl_batcher.so var/casew/libsdl_batcher.so
