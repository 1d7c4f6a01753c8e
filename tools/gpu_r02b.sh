set -u
mkdir -p gpurun_out/r02b
SDL_LIB=build/stamps/libsdl_batcher.so timeout -k 10 120 python tools/wp_stamps.py mlm 64 > gpurun_out/r02b/stamps_mlm.txt 2>&1 || exit $?
timeout -k 10 600 tools/ablate.sh > gpurun_out/r02b/ablate.txt 2>&1 || exit $?
cp gpurun_out/ablate.txt gpurun_out/r02b/ablate_stages.txt
