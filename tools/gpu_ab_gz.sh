#!/bin/bash
# A/B of inflate builds on the bench's gzip leg (256 MiB arena: ~4,100 BGZF members).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abgz
for lib in "$@"; do
  SDL_LIB=$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --gz --no-cpu-baseline --arena-mib ${MIB:-256} > gpurun_out/abgz/b.json 2> gpurun_out/abgz/b.err || { tail -20 gpurun_out/abgz/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/abgz/b.json'))['provider_gzip']; print('$lib', d['inflated_MBps'], d['ms'], d['members'])"
done
