#!/usr/bin/env python3
"""Diagnostic: t5 ids of held-out records on the device (the full corpus in one arena, as
tests/test_gpu_full_size.py runs it) against the oracle; prints each differing record's first
mismatch with the pieces around it.  python tools/debug_t5_record.py [record ...]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

import oracle_lib  # noqa: E402
from streaming_data_loader_amd import native  # noqa: E402
from test_gpu_full_size import device_ids  # noqa: E402

recs = [json.loads(l)["text"] for l in open(os.path.join(REPO, "tests", "golden", "heldout_records.jsonl"))]
blobs = [r.encode("utf-8") for r in recs]
got = device_ids(torch, blobs, "t5", native.T5_PROXY_TOKENIZER)
vocab = [p for p, _ in json.load(open(native.T5_PROXY_TOKENIZER))["model"]["vocab"]]
tok = oracle_lib.T5Tok()
want_recs = [int(a) for a in sys.argv[1:]] or range(len(recs))
for r in want_recs:
    want = [1] + tok.encode(recs[r]) + [1]
    if got[r] == want:
        continue
    k = next((i for i in range(min(len(got[r]), len(want))) if got[r][i] != want[i]), min(len(got[r]), len(want)))
    print(f"record {r}: {len(got[r])} vs {len(want)} ids, first difference at {k}")
    print("  device:", [vocab[i] if i < len(vocab) else i for i in got[r][max(0, k - 6):k + 8]])
    print("  oracle:", [vocab[i] if i < len(vocab) else i for i in want[max(0, k - 6):k + 8]])
