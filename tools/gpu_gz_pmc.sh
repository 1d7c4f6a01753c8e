#!/bin/bash
# Instruction mix and wait cycles of k_inflate (two --pmc passes, kernel trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/gzpmc; rm -rf $O; mkdir -p $O
B="python3 bench.py --steps 1 --warmup 0 --gz --no-cpu-baseline --arena-mib 64"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $O/a -o run -- $B > $O/a.out 2> $O/a.err || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA \
  --kernel-trace --output-format csv -d $O/b -o run -- $B > $O/b.out 2> $O/b.err || exit $?
for p in a b; do
  f=$(find $O/$p -name '*counter_collection.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(float)
for r in rows:
    if "k_inflate" in r.get("Kernel_Name", ""):
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(acc.items()):
    print(f"{k:24s} {v:16.0f}")
PY
done
