#!/bin/bash
# Device gzip inflate: parity tests, then the bench's provider_gzip leg and its rocprof kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/gz
timeout -k 10 300 python -u -m pytest tests/test_inflate.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/gz/test.log 2>&1 || { tail -40 gpurun_out/gz/test.log; exit 1; }
tail -3 gpurun_out/gz/test.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --gz --no-cpu-baseline --arena-mib ${MIB:-64} \
    > gpurun_out/gz/bench.json 2> gpurun_out/gz/bench.err || { tail -30 gpurun_out/gz/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/gz/bench.json')); print(json.dumps(d['provider_gzip'], indent=1))"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gz/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --gz \
    --no-cpu-baseline --arena-mib 64 > gpurun_out/gz/prof.json 2> gpurun_out/gz/prof.err || { tail -20 gpurun_out/gz/prof.err; exit 1; }
f=$(find gpurun_out/gz/prof -name '*kernel_stats.csv' | head -1)
grep -E "Name|k_inflate|k_gz|k_json|k_wordpiece" "$f" | cut -c1-200
