#!/bin/bash
# held-out clm at HEAD: bench (stage times), BPE phase stamps, rocprof kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04j; mkdir -p $O; export TMPDIR=/tmp
for c in fixture heldout; do
  timeout -k 10 300 python -u bench.py --task clm --corpus $c --steps 10 --warmup 2 --no-cpu-baseline --soak-s 0 > $O/clm_$c.json 2> $O/clm_$c.err || exit 1
  python -c "import json; d=json.load(open('$O/clm_$c.json')); print('clm $c', d['value'], d['stage_ms'])"
done
SDL_LIB=var/stamps/libsdl_batcher.so timeout -k 10 200 python tools/wp_stamps.py clm 64 heldout > $O/stamps_clm_heldout.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/stamps_clm_heldout.txt | tail -30
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_clm_heldout -o run --output-format csv -- python3 bench.py --task clm --corpus heldout --steps 5 --warmup 2 --no-cpu-baseline --soak-s 0 > $O/prof.json 2> $O/prof.err || exit 1
f=$(find $O/prof_clm_heldout -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 "$f" | head -12
