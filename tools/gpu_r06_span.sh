set -u
O=gpurun_out/r06b; mkdir -p $O; export TMPDIR=/tmp
SDL_LIB=var/stamps/libsdl_batcher.so timeout -k 10 150 python tools/uni_stamps.py 64 fixture > $O/stamps_old.txt 2>&1 || exit 11
SDL_LIB=var/r05head/libsdl_batcher.so timeout -k 10 200 python bench.py --task span --steps 10 --warmup 2 --no-cpu-baseline > $O/span_old.json 2> $O/span_old.err || exit 12
OUT=r06b/tests bash tools/gpu_tests.sh tests/test_gpu_span.py tests/test_gpu_t5_kat.py || exit 13
SDL_LIB=var/stamps_new/libsdl_batcher.so timeout -k 10 150 python tools/uni_stamps.py 64 fixture > $O/stamps_new.txt 2>&1 || exit 14
timeout -k 10 200 python bench.py --task span --steps 10 --warmup 2 --no-cpu-baseline > $O/span_new.json 2> $O/span_new.err || exit 15
