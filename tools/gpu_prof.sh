#!/bin/bash
# rocprof kernel stats of one bench configuration per library: gpurun_out/${OUT:-prof}/<name>/
#   TASK=span CORPUS=fixture bash tools/gpu_prof.sh lib1 lib2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-prof}; mkdir -p $O; export TMPDIR=/tmp
for lib in "$@"; do
  name=$(basename $(dirname $lib))_${TASK:-mlm}_${CORPUS:-fixture}
  SDL_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o run -- python3 bench.py --task ${TASK:-mlm} --corpus ${CORPUS:-fixture} --steps 10 --warmup 2 --no-cpu-baseline --soak-s 0 ${BENCH_ARGS:-} > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
  find $O/$name -name '*kernel_trace.csv' -delete
  f=$(find $O/$name -name '*kernel_stats.csv' | head -1)
  echo "== $name"; cut -d, -f1-4 "$f" | head -8
done
