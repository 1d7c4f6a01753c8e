#!/bin/bash
# r03: rand-mode / span / inflate GPU tests; Unigram A/B (r02 lib, HEAD, adj8) with kernel stats and PMC.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03d; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rand_mode.py tests/test_inflate_fuzz.py tests/test_gpu_span.py -m gpu -v --timeout 120 --timeout-method thread -rf > $O/pytest.log 2>&1
echo "[pytest] exit $?" | tee -a $O/steps.log; tail -1 $O/pytest.log
bash tools/gpu_measure.sh "mlm_r1:--rng-mode 1 --no-cpu-baseline" || exit $?
CORPORA=fixture TASK=span bash tools/gpu_ab.sh var/old/libsdl_batcher.so streaming_data_loader_amd/libsdl_batcher.so var/adj8/libsdl_batcher.so || exit $?
for v in old head; do
  lib=var/old/libsdl_batcher.so; [ $v = head ] && lib=streaming_data_loader_amd/libsdl_batcher.so
  SDL_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 bench.py --task span --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_$v.out 2> $O/prof_$v.err || exit $?
  SDL_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_$v -o run -- python3 bench.py --task span --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_$v.out 2> $O/pmc_$v.err || exit $?
  echo "[$v] profiled" | tee -a $O/steps.log
done
