#!/bin/bash
# End-to-end frames for mlm incl. the gzip (BGZF) input variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/e2e
for t in ${TASKS:-mlm}; do
  timeout -k 10 400 python3 bench.py --task $t --e2e-frames --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/e2e/$t.json 2> gpurun_out/e2e/$t.err || { tail -20 gpurun_out/e2e/$t.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/e2e/$t.json'))['end_to_end_frames']
print('$t seq', d['MBps'], 'gz', d['from_gzip'], 'd2h', d['d2h_only']['text_MBps_bound'], 'pipe', max(p['MBps'] for p in d['pipelined']))"
done
