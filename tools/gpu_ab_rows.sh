set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py tests/test_gpu_rand_mode.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/t.log 2>&1 || { tail -30 gpurun_out/ab/t.log; exit 1; }
tail -1 gpurun_out/ab/t.log
P=build/var/prev/libsdl_batcher.so; C=streaming_data_loader_amd/libsdl_batcher.so
CORPORA=fixture TASK=mlm tools/gpu_ab.sh $P $C $P $C || exit 1
CORPORA=fixture TASK=clm tools/gpu_ab.sh $P $C || exit 1
CORPORA=fixture TASK=span tools/gpu_ab.sh $C build/var/dpg4/libsdl_batcher.so build/var/dpg16/libsdl_batcher.so build/var/w2/libsdl_batcher.so build/var/w4/libsdl_batcher.so || exit 1
