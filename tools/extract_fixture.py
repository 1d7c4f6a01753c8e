#!/usr/bin/env python3
"""Copy the reference's own masking-test input (`data/test.json.gz`, used by
`rust/src/tasks/masking/masking_cases.rs:13-21`) into a committed fixture.

Only the `text` field of each JSON line is kept, in file order, exactly as the
reference's provider extracts it (`rust/src/provider/provider_util.rs:61-64`:
lines whose `text` is not a string are skipped).  Run in the build container.
"""
import gzip, json, os, sys
src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/data/test.json.gz"
dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "test_records.jsonl")
n = 0
with gzip.open(src, "rt", encoding="utf-8") as f, open(dst, "w", encoding="utf-8") as o:
    for line in f:
        v = json.loads(line)
        t = v.get("text")
        if isinstance(t, str):
            o.write(json.dumps({"text": t}, ensure_ascii=False) + "\n")
            n += 1
print(n, "records ->", dst)
