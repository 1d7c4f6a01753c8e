#!/bin/bash
# mlm in both RNG modes (and rng_mode 1 variants: SDL_RAND_REC0=0, extra libraries as arguments),
# fixture corpus, then rocprof kernel stats of rng_mode 1.  Output: gpurun_out/${OUT:-rng}/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-rng}; mkdir -p $O; export TMPDIR=/tmp
run() {  # run NAME ENV... -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --soak-s 0 $BARGS > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['ms_per_step'], d.get('stage_ms'))" | tee -a $O/summary.txt
}
BARGS="--rng-mode 0" run r0 X=1
BARGS="--rng-mode 1" run r1 X=1
BARGS="--rng-mode 1" run r1_norec0 SDL_RAND_REC0=0
for lib in "$@"; do BARGS="--rng-mode 1" run r1_$(basename $(dirname $lib)) SDL_LIB=$lib; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r1 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --rng-mode 1 --no-cpu-baseline --soak-s 0 > $O/prof_r1.out 2> $O/prof_r1.err || { tail -5 $O/prof_r1.err; exit 1; }
find $O/prof_r1 -name '*kernel_trace.csv' -delete
f=$(find $O/prof_r1 -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 "$f" | head -16
