#!/bin/bash
# Host-path measurements for DESIGN.md: record path + channel (--e2e), JSON
# filter (--json), JSON lines -> frames sequential and chunked (--e2e-frames),
# device frames (--frames), all for mlm at 64 MiB.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-host}; mkdir -p $O
export TMPDIR=/tmp
A="--task ${TASK:-mlm} --steps 3 --warmup 1 --arena-mib 64 --no-cpu-baseline"
timeout -k 10 300 python bench.py $A --e2e > $O/e2e.json 2> $O/e2e.err || exit $?
timeout -k 10 300 python bench.py $A --json > $O/json.json 2> $O/json.err || exit $?
timeout -k 10 300 python bench.py $A --e2e-frames > $O/e2e_frames.json 2> $O/e2e_frames.err || exit $?
timeout -k 10 300 python bench.py --task ${TASK:-mlm} --steps 5 --warmup 2 --no-cpu-baseline --frames > $O/frames.json 2> $O/frames.err || exit $?
echo done
