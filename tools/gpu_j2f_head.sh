#!/bin/bash
# sdl_json_to_frames: first-chunk divisor sweep (SDL_J2F_HEAD), mlm 64 MiB.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/j2f
for h in 4 8 16 32; do
  SDL_J2F_HEAD=$h timeout -k 10 300 python3 bench.py --e2e-frames --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/j2f/h$h.json 2> gpurun_out/j2f/h$h.err || { tail -5 gpurun_out/j2f/h$h.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/j2f/h$h.json'))['end_to_end_frames']
print('head $h', [(p['chunk_MiB'], p['input'], p['MBps']) for p in d['pipelined']], 'bound', d['d2h_only']['text_MBps_bound'])"
done
