#!/usr/bin/env python3
"""Timeline of the last K dispatches of a rocprofv3 --kernel-trace CSV (start offset, duration,
queue/stream id), relative to the first of them: python tools/trace_timeline.py TRACE.csv [K]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-k:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
    print(f"{s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f} us  q={q:>3}  {r['Kernel_Name'][:70]}")
