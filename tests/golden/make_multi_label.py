#!/usr/bin/env python3
"""Generate the multi-label golden vectors under tests/golden/.

  multi_label.arrow        Arrow IPC stream with the reference's multi-label
                           schema (MultiArrowGenerator, rust/src/tasks/multi_label/
                           multi_arrow.rs:36-41: `sentence: utf8`,
                           `labels: list<int64>`): the 50 fixture records of
                           data/test.json.gz, each with 0-4 distinct labels out
                           of 9 drawn with seed 42,
                           written as 3 record batches.
  multi_label_s128_b8.npz  every batch SimpleBatcher emits over that stream at
                           seq_len=128, batch=8, then the end-of-stream flush
                           (simple_batcher.rs:35-53 + BertData MultiLabel,
                           bert_data.rs:55-89), from the pure-Python restatement
                           below with ids from the HF `tokenizers` binding.

Run in the build container:  python tests/golden/make_multi_label.py
"""
import json
import os
import sys

import numpy as np
import pyarrow as pa
from tokenizers import Tokenizer

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
ASSET = os.path.join(REPO, "streaming_data_loader_amd", "assets", "bert_proxy", "tokenizer.json")
NUMBER_LABELS = 9


def records():
    with open(os.path.join(HERE, "test_records.jsonl"), encoding="utf-8") as f:
        return [json.loads(l)["text"] for l in f]


def seeded_labels(n, seed=42):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        k = int(rng.integers(0, 5))
        out.append(sorted(int(x) for x in rng.choice(NUMBER_LABELS, size=k, replace=False)))
    return out


class PySimpleBatcher:
    """SimpleBatcher + BertData(MultiLabel) restated in Python."""

    def __init__(self, tok, B, S, NL):
        self.tok, self.B, self.S, self.NL = tok, B, S, NL
        self.cls, self.sep = tok.token_to_id("[CLS]"), tok.token_to_id("[SEP]")
        self.batch = self.new_batch()

    def new_batch(self):
        B, S = self.B, self.S
        return {"input_ids": np.zeros((B, S), np.int32), "attention_mask": np.ones((B, S), np.int32),
                "token_type_ids": np.zeros((B, S), np.int32), "labels": np.zeros((B, self.NL), np.float32),
                "index": 0}

    def create_sync_batch(self, text, labels):
        # TokenizerWrapper::encode_simple -> encode_mask framing (tokenizer_wrapper.rs:101-116)
        ids = [self.cls] + self.tok.encode(text, add_special_tokens=True).ids + [self.sep, self.sep]
        b, S, r = self.batch, self.S, self.batch["index"]
        l = min(S, len(ids))
        b["input_ids"][r, :l] = ids[:l]
        if len(ids) < S:
            b["attention_mask"][r, S - len(ids):] = 0
        for x in labels:
            b["labels"][r, x] = 1.0
        b["index"] += 1
        if b["index"] == self.B:
            return self.get_working_batch()
        return None

    def get_working_batch(self):
        old, self.batch = self.batch, self.new_batch()
        return old


def main():
    recs = records()
    labels = seeded_labels(len(recs))
    table = pa.table({"sentence": pa.array(recs, pa.utf8()),
                      "labels": pa.array(labels, pa.list_(pa.int64()))})
    with pa.OSFile(os.path.join(HERE, "multi_label.arrow"), "wb") as f:
        with pa.ipc.new_stream(f, table.schema) as w:
            for batch in table.to_batches(max_chunksize=20):
                w.write_batch(batch)
    tok = Tokenizer.from_file(ASSET)
    pb = PySimpleBatcher(tok, 8, 128, NUMBER_LABELS)
    out = []
    for t, l in zip(recs, labels):
        b = pb.create_sync_batch(t, l)
        if b is not None:
            out.append(b)
    out.append(pb.get_working_batch())
    arrs = {}
    for i, b in enumerate(out):
        for k in ("input_ids", "attention_mask", "token_type_ids", "labels"):
            arrs[f"b{i}_{k}"] = b[k]
        arrs[f"b{i}_rows"] = np.int32(b["index"])
    arrs["n_batches"] = np.int32(len(out))
    np.savez_compressed(os.path.join(HERE, "multi_label_s128_b8.npz"), **arrs)
    print(f"{len(out)} multi-label batches (last has {out[-1]['index']} rows)", file=sys.stderr)


if __name__ == "__main__":
    main()
