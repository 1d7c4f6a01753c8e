#!/bin/bash
# rocprofv3 kernel-trace summary of one bench task: tools/gpu_prof_task.sh TASK [LIB]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/prof_$1${2:+_$(basename $(dirname $2))}
SDL_LIB=${2:-streaming_data_loader_amd/libsdl_batcher.so} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out -o run --output-format csv -- python3 bench.py --task $1 --steps 5 --warmup 2 --no-cpu-baseline > $out.json 2> $out.err
rc=$?
python3 -c "
import csv,sys
for r in csv.DictReader(open('$out/run_kernel_stats.csv')):
    print('$out', r['Name'].split('(')[0][:40], r['Calls'], round(float(r['AverageNs'])/1e6, 4))" 2>/dev/null | head -8
exit $rc
