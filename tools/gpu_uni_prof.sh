set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/uni2
SDL_LIB=build/stamps/libsdl_batcher.so timeout -k 10 120 python tools/wp_stamps.py span 64 > gpurun_out/uni2/stamps_span.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/uni2/prof -o run --output-format csv -- python3 bench.py --task span --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/uni2/prof.json 2> gpurun_out/uni2/prof.err || exit $?
