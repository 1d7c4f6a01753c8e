#!/bin/bash
# rng_mode 1 beside the tokenizer: parity, then mlm bench in both RNG modes, rocprof stats of mode 1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-r04b}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rand_mode.py tests/test_multi_shard.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/test.log 2>&1; rc=$?; tail -2 $O/test.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/test.log | head -20; exit $rc; }
for m in 1 0; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --rng-mode $m --no-cpu-baseline --soak-s 0 > $O/bench_mlm_r$m.json 2> $O/bench_mlm_r$m.err || { tail -20 $O/bench_mlm_r$m.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_mlm_r$m.json')); print('rng', $m, d['value'], d['ms_per_step'], d.get('stages_ms'))"
done
SDL_RAND_SPEC=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --rng-mode 1 --no-cpu-baseline --soak-s 0 > $O/bench_mlm_r1_nospec.json 2> $O/bench_mlm_r1_nospec.err || exit 1
python -c "import json; d=json.load(open('$O/bench_mlm_r1_nospec.json')); print('rng 1 nospec', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r1 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --rng-mode 1 --no-cpu-baseline --soak-s 0 > $O/prof_r1.json 2> $O/prof_r1.err || { tail -20 $O/prof_r1.err; exit 1; }
f=$(find $O/prof_r1 -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 "$f" | head -20
