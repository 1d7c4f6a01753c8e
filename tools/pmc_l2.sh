#!/bin/bash
# L2 hit/miss counters of one bench task's kernels: tools/pmc_l2.sh TASK
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc_l2_$1 -o run -- python3 bench.py --task $1 --steps 1 --warmup 1 --arena-mib 64 --no-cpu-baseline > gpurun_out/pmc_l2_$1.out 2> gpurun_out/pmc_l2_$1.err
rc=$?
python3 - "$1" <<'PY'
import csv, glob, sys, collections
f = glob.glob(f"gpurun_out/pmc_l2_{sys.argv[1]}/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(float)
for r in csv.DictReader(open(f[0])):
    acc[(r["Kernel_Name"].split("(")[0][:40], r["Counter_Name"])] += float(r["Counter_Value"])
for k, v in sorted(acc.items()):
    print(k, v)
PY
exit $rc
