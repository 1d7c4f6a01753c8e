#!/usr/bin/env python3
"""Diagnostic: one large gzip member (the reference's input shape) through
sdl_gzip_inflate_device's chunked path; with SDL_GZ_DEBUG=1 the library prints
its phase times.  python tools/gz_single.py [JSON MiB] [level] [corpus]"""
import json
import os
import sys
import time
import zlib

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from streaming_data_loader_amd.device import DeviceBatcher  # noqa: E402

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
level = int(sys.argv[2]) if len(sys.argv) > 2 else 6
corpus = sys.argv[3] if len(sys.argv) > 3 else "fixture"
records = bench.corpus_records(corpus)
_, _, order = bench.build_arena(records, mib << 20, seed=0x5D1B)
lines, size = [], 0
for i, k in enumerate(order):
    ln = json.dumps({"id": i, "title": f"t{i}", "text": records[k]}).encode() + b"\n"
    lines.append(ln)
    size += len(ln)
    if size >= mib << 20:
        break
buf = b"".join(lines)
co = zlib.compressobj(level, zlib.DEFLATED, 31)
gz = co.compress(buf) + co.flush()
a = np.zeros(len(gz) + 32, np.uint8)
a[:len(gz)] = np.frombuffer(gz, np.uint8)
d = torch.from_numpy(a).cuda()
off = torch.from_numpy(np.array([0, len(gz)], np.int64)).cuda()
db = DeviceBatcher(batch_size=8, sequence_length=128)
for it in range(4):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = db.gzip_inflate(d.data_ptr(), len(gz), off.data_ptr(), 1)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"[gz single] {corpus} level {level}: {len(buf) / 1e6:.1f} MB JSON, {len(gz) / 1e6:.1f} MB member: "
          f"{dt * 1e3:.2f} ms = {len(buf) / dt / 1e9:.2f} GB/s", file=sys.stderr, flush=True)
assert int(out.out_bytes) == len(buf) and int(out.n_bad) == 0
