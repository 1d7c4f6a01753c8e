#!/bin/bash
# per-record push latency: timing, host laps, kernel trace of the launches per push
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/push${PUSH_TAG:-}; mkdir -p $O
for t in mlm clm span; do
  timeout -k 10 120 python tools/push_latency.py --task $t --records 2000 | tee -a $O/lat.txt || exit $?
done
SDL_HOST_TIMING=1 timeout -k 10 120 python tools/push_latency.py --records 8 > $O/laps.txt 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/push_latency.py --records 300 > $O/prof.out 2>&1 || exit $?
