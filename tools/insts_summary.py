#!/usr/bin/env python3
"""Per-wave instruction mix of the kernels in gpurun_out/insts (tools/gpu_insts.sh).

    python tools/insts_summary.py [gpurun_out/insts] [min_waves]
"""
import csv
import glob
import os
import sys
from collections import defaultdict

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/insts"
min_waves = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
libs = dict(l.split(" ", 1) for l in open(os.path.join(src, "libs.txt")).read().split("\n") if l)
for i, lib in sorted(libs.items()):
    vals = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(src, f"l{i}", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"].split("(")[0].replace("void ", "")
                vals[k][row["Counter_Name"]] += float(row["Counter_Value"])
    for k, c in vals.items():
        w = c.get("SQ_WAVES", 0)
        if w < min_waves:
            continue
        mix = " ".join(f"{n[9:]} {c.get(n, 0) / w:.0f}" for n in
                       ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SMEM"))
        print(f"{lib:50s} {k[:28]:28s} waves {w:.0f} {mix} cycles/wave {c.get('GRBM_GUI_ACTIVE', 0) / 8 * 256 / w:.0f}")
