#!/usr/bin/env python3
"""Average kernel durations (ms) from rocprofv3 *kernel_stats.csv files: kstats.py DIR..."""
import csv
import glob
import os
import re
import sys

for d in sys.argv[1:]:
    for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)):
        rows = list(csv.DictReader(open(f)))
        out = []
        for r in rows:
            name = re.sub(r"\(.*", "", r["Name"]).replace("sdl::", "").replace("void ", "")
            out.append((name, int(r["Calls"]), float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
        steps = max((c for n, c, a, t in out if "chunks" in n), default=1)
        print(f"== {d}  ({steps} calls of the tokenizer)")
        for n, c, a, t in sorted(out, key=lambda x: -x[3])[:9]:
            print(f"   {n:38s} calls {c:5d} avg {a:8.4f} ms  per-step {t / steps:8.4f} ms")
