#!/usr/bin/env python3
"""Generate the gpt2 (byte-level BPE) golden vectors under tests/golden/.

  gpt2_ids.json     Tokenizer.encode(text, add_special_tokens=True).ids with the
                    proxy gpt2 asset (tools/make_proxy_gpt2.py) from the HF
                    `tokenizers` binding (0.22.2 here; the reference pins the
                    same project's crate at 0.13.1 and calls it at
                    rust/src/tokenizer/tokenizer_holder.rs:22) for the fixture
                    records, regex edge cases (contractions, whitespace runs,
                    prefix spaces, <|endoftext|>) and seeded random strings.
  clm_s128_b8.npz   every batch GenTokenizer + GptData emits on the fixture
                    stream at seq_len=128, batch=8, then the end-of-stream
                    flush (gen_batcher.rs:69-98, gpt_data.rs:15-45), from the
                    pure-Python restatement below.

Run in the build container:  python tests/golden/make_gpt2_goldens.py
"""
import json
import os
import random
import sys

import numpy as np
from tokenizers import Tokenizer

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
ASSET = os.path.join(REPO, "streaming_data_loader_amd", "assets", "gpt2_proxy", "tokenizer.json")


def records():
    with open(os.path.join(HERE, "test_records.jsonl"), encoding="utf-8") as f:
        return [json.loads(l)["text"] for l in f]


def edge_cases():
    return [
        "", " ", "  ", "   x", "a  ", "a \n b", "a\n\nb", "\n's", " 's", "  's", "''s", "!'s", "it's'd",
        "'S 'T 'RE", "'s'S'll've're'm'd't", "'l 'lx 'r 'v", "x'", "'", "' s", "don't won't y'all",
        "12.5e3 1٣ ²³ Ⅻ", "\t\t\nfoo\r\n", " nbsp em　ideo", "\x0b\x0c\x1c\x1d",
        "<|endoftext|>", "<|endoftext|><|endoftext|>", "a<|endoftext|> b", "x <|endoftext|>  y", "<|endof",
        "ÄÖÜ äöü ß 中文 日本語 😀😀 🇩🇪", "café naïve résumé", "​‍zw", "a" * 300, " " * 70 + "x",
        "=" * 90, "1234567890" * 8, "https://en.wikipedia.org/wiki/Foo_(bar)?a=1&b=2",
    ]


def random_strings(n, seed=11):
    rng = random.Random(seed)
    alpha = list("abcdefghijklmnopqrstuvwxyz ABCXYZ     \n\n\t'''sltrevmd0123456789!,.;:?-()[]") + \
        ["é", "ß", "İ", "Ａ", "中", "😀", " ", "　", "٣", "<|endoftext|>", "\r\n"]
    return ["".join(rng.choice(alpha) for _ in range(rng.randint(0, 60))) for _ in range(n)]


class PyGpt:
    """GenTokenizer(chunk=true) + GptData restated in Python."""

    def __init__(self, tok, B, S):
        self.tok, self.B, self.S = tok, B, S
        self.eos = tok.token_to_id("<|endoftext|>")
        self.store = [self.new_batch()]

    def new_batch(self):
        B, S = self.B, self.S
        return {"input_ids": np.zeros((B, S), np.int32), "attention_mask": np.ones((B, S), np.int32),
                "labels": np.full((B, S), -100, np.int32), "index": 0}

    def put(self, b, ids):
        S, r = self.S, b["index"]
        b["input_ids"][r, :len(ids)] = ids
        b["labels"][r, :] = b["input_ids"][r, :]
        if len(ids) < S:
            b["labels"][r, S - len(ids):] = -100
            b["attention_mask"][r, S - len(ids):] = 0
        b["index"] += 1

    def create_sync_batch(self, text):
        ids = [self.eos] + self.tok.encode(text, add_special_tokens=True).ids + [self.eos]
        if len(ids) < 64:
            return None
        for off in range(0, len(ids), self.S):
            self.put(self.store[-1], ids[off:off + self.S])
            if self.store[-1]["index"] == self.B:
                self.store.append(self.new_batch())
        if self.store[0]["index"] == self.B:
            return self.store.pop(0)
        return None

    def get_working_batch(self):
        return self.store.pop(0) if self.store else None


def main():
    tok = Tokenizer.from_file(ASSET)
    recs = records()
    cases = [{"text": t, "ids": tok.encode(t, add_special_tokens=True).ids}
             for t in recs + edge_cases() + random_strings(400)]
    with open(os.path.join(HERE, "gpt2_ids.json"), "w", encoding="utf-8") as f:
        json.dump({"generator": "tokenizers " + __import__("tokenizers").__version__,
                   "asset": "streaming_data_loader_amd/assets/gpt2_proxy/tokenizer.json",
                   "n_fixture_records": len(recs), "cases": cases}, f, ensure_ascii=False)
    pg = PyGpt(tok, 8, 128)
    out = [b for b in (pg.create_sync_batch(t) for t in recs) if b is not None]
    out.append(pg.get_working_batch())
    arrs = {}
    for i, b in enumerate(out):
        for k in ("input_ids", "attention_mask", "labels"):
            arrs[f"b{i}_{k}"] = b[k]
        arrs[f"b{i}_rows"] = np.int32(b["index"])
    arrs["n_batches"] = np.int32(len(out))
    np.savez_compressed(os.path.join(HERE, "clm_s128_b8.npz"), **arrs)
    print(f"{len(cases)} id cases, {len(out)} clm batches (last has {out[-1]['index']} rows)", file=sys.stderr)


if __name__ == "__main__":
    main()
