#!/bin/bash
# r04: rand walk with two interleaved ChaCha12 blocks -- rng_mode 1 parity, A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04s; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rand_mode.py tests/test_multi_shard.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1; rc=$?; tail -1 $O/test.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/test.log | head; exit $rc; }
for lib in var/walk1/libsdl_batcher.so streaming_data_loader_amd/libsdl_batcher.so; do
  SDL_LIB=$lib timeout -k 10 200 python bench.py --task mlm --rng-mode 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/b.json 2>>$O/b.err || exit $?
  python -c "import json;d=json.load(open('$O/b.json'));print('mlm rng1 $lib', d['value'], d['stage_ms'])" | tee -a $O/ab.txt
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --task mlm --rng-mode 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/prof.out 2>&1 || exit $?
find $O/prof -name '*kernel_trace.csv' -delete
