#!/bin/bash
# BPE phase stamps (var/stamps) on both corpora + held-out clm rocprof kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/bpe_stamps; mkdir -p $O; export TMPDIR=/tmp
for c in fixture heldout; do
  SDL_LIB=var/stamps/libsdl_batcher.so timeout -k 10 150 python tools/wp_stamps.py clm 64 $c > $O/clm_$c.txt 2>&1 || exit $?
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --task clm --corpus heldout --no-cpu-baseline > $O/prof.out 2>&1 || exit $?
find $O/prof -name '*kernel_trace.csv' -delete
grep -h -v amdgpu.ids $O/clm_*.txt | grep -i "stamp\|long" | head -40
