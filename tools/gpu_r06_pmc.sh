#!/bin/bash
# Instruction mix + wait cycles per wave of the span kernels for libraries given as arguments
# (64 MiB fixture arena; one --pmc pass per counter group).  Output: gpurun_out/r06pmc/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06pmc}; mkdir -p $O
i=0
for lib in "$@"; do
  i=$((i+1)); echo "$i $lib" >> $O/libs.txt
  for g in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT"; do
    tag=$(echo $g | cut -c10-20 | tr ' ' _)
    SDL_LIB=$lib timeout -k 10 120 rocprofv3 --pmc $g --kernel-trace --output-format csv -d $O/l$i/$tag -o run -- python3 bench.py --task ${TASK:-span} --steps 2 --warmup 1 --arena-mib 64 --no-cpu-baseline --no-heldout --soak-s 0 --corpus ${CORPUS:-fixture} > $O/l$i.$tag.out 2> $O/l$i.$tag.err || exit $?
  done
done
python3 - "$O" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
src = sys.argv[1]
libs = dict(l.split(" ", 1) for l in open(os.path.join(src, "libs.txt")).read().split("\n") if l)
for i, lib in sorted(libs.items()):
    vals = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(src, f"l{i}", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0].replace("void ", "")
            vals[k][row["Counter_Name"]] += float(row["Counter_Value"])
    for k, c in vals.items():
        w = c.get("SQ_WAVES", 0) / 2  # (two passes each counted SQ_WAVES)
        if w < 1000:
            continue
        print(lib, k, "waves", int(w), " ".join(f"{n}={c[n] / w:.0f}" for n in sorted(c) if n != "SQ_WAVES"))
PY
