#!/bin/bash
# rng_mode 1: speculation guess sweep (bench only)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-r04e}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rand_mode.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1; rc=$?; tail -1 $O/test.log; [ $rc -eq 0 ] || exit $rc
for cfg in "1 40" "1 50" "1 60" "1 80" "0 40"; do
  set -- $cfg
  SDL_RAND_SPEC=$1 SDL_RAND_SPEC_BPC10=$2 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --rng-mode 1 --no-cpu-baseline --soak-s 0 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || exit 1
  python -c "import json; d=json.load(open('$O/b_$1_$2.json')); print('spec $1 bpc10 $2', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --rng-mode 0 --no-cpu-baseline --soak-s 0 > $O/b_philox.json 2> $O/b_philox.err || exit 1
python -c "import json; d=json.load(open('$O/b_philox.json')); print('philox', d['value'], d['ms_per_step'])"
