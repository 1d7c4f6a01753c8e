#!/usr/bin/env python3
"""Generate the committed golden vectors under tests/golden/.

Run in the build container (needs the HF `tokenizers` binding, 0.22.2 here):

  bert_ids.json     token ids of Tokenizer.encode(text, add_special_tokens=True)
                    with the proxy bert-base-uncased asset, for every record of
                    the reference fixture (data/test.json.gz) plus edge cases
                    and seeded random Unicode strings.  `tokenizers` is the same
                    project as the crate the reference calls at
                    rust/src/tokenizer/tokenizer_holder.rs:22 (pinned 0.13.1 in
                    rust/Cargo.lock, not vendored).
  mlm_s128_b8.npz   every batch the reference MLM Batcher emits on the fixture
                    stream at the reference's CPU config (seq_len=128, batch=8,
                    BASELINE.json configs[0]) under the seeded RNG contract,
                    followed by the end-of-stream flush.  Produced by the pure
                    Python restatement below (ids from `tokenizers` itself), so
                    it checks the C oracle's batching/masking independently.
"""
import json
import os
import random
import sys

import numpy as np
from tokenizers import Tokenizer

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
ASSET = os.path.join(REPO, "streaming_data_loader_amd", "assets", "bert_proxy", "tokenizer.json")

M32 = 0xFFFFFFFF


def philox4x32_10(c, k0, k1):
    c = list(c)
    for _ in range(10):
        p0 = 0xD2511F53 * c[0]
        p1 = 0xCD9E8D57 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k0) & M32, p1 & M32, ((p0 >> 32) ^ c[3] ^ k1) & M32, p0 & M32]
        k0 = (k0 + 0x9E3779B9) & M32
        k1 = (k1 + 0xBB67AE85) & M32
    return c


def mlm_keys(seed, record, chunk, S):
    keys = []
    for q in range((S + 3) // 4):
        keys += philox4x32_10([q, chunk, record & M32, record >> 32], seed & M32, seed >> 32)
    return keys[:S]


def records():
    with open(os.path.join(HERE, "test_records.jsonl"), encoding="utf-8") as f:
        return [json.loads(l)["text"] for l in f]


def edge_cases():
    cases = [
        "", " ", "\t\n\r", "\x00", "a\x00b", "�", "x�y", "zw​sp", "soft­hyphen",
        "[SEP]", "x[MASK]y", "[sep]", "[[SEP]]", "[SEP", "[CLS][SEP][PAD][UNK][MASK]", "a [PAD] b",
        "İstanbul", "Ångström", "ﬁle", "straße", "naïve café",
        "中文字", "한국어", "日本語のテキスト",
        "a" * 100, "a" * 101, "é" * 100, "é" * 101, "é", "́abc", "\x0b\x0cvt ff",
        "nbsp here", "\U0001f600\U0001f44d emoji", "Привет мир",
        "άλφα", "العربية", "हिन्दी",
        "∑x≤y", "$100.00", "don't", "U.S.A.", "3.14159", "https://example.com/a_b?c=d&e=f",
        "".join(chr(c) for c in range(32, 127)), "tokenization internationalization",
        "supercalifragilisticexpialidocious" * 3, "x" + "​" * 200 + "y", "a　b",
        " line para", "ᅠᅟ", "\U00020000\U0002a6d6", "豈﫿",
        "ab️cd", "\U000e0001tag", "½ ⑴ Ⅰ", ";·",
    ]
    rng = random.Random(0x5D1B)
    ranges = [(0x20, 0x7E), (0x20, 0x7E), (0x20, 0x7E), (0xA0, 0x24F), (0x300, 0x36F), (0x370, 0x3FF),
              (0x400, 0x4FF), (0x590, 0x6FF), (0x900, 0x97F), (0x1100, 0x11FF), (0x2000, 0x206F),
              (0x2100, 0x22FF), (0x3000, 0x30FF), (0x4E00, 0x4F00), (0xAC00, 0xAD00), (0xF900, 0xFAFF),
              (0xFE00, 0xFFFF), (0x1F300, 0x1F6FF), (0x20000, 0x20100), (0xE0000, 0xE007F), (0x0, 0x1F)]
    for _ in range(300):
        n = rng.randint(1, 60)
        s = []
        for _ in range(n):
            lo, hi = rng.choice(ranges)
            c = rng.randint(lo, hi)
            if 0xD800 <= c <= 0xDFFF:
                c = 0x41
            s.append(chr(c))
            if rng.random() < 0.15:
                s.append(" ")
            if rng.random() < 0.02:
                s.append(rng.choice(["[SEP]", "[MASK]", "[CLS]", "[PAD]", "[UNK]"]))
        cases.append("".join(s))
    return cases


class PyBatcher:
    """GenTokenizer(chunk=true) + BertData(Mask) restated in Python
    (rust/src/tasks/gen_batcher.rs:44-98, rust/src/models/bert_data.rs:27-93)."""

    def __init__(self, tok, B, S, mask_length, mask_id, seed):
        self.tok, self.B, self.S = tok, B, S
        self.mask_length, self.mask_id, self.seed = mask_length, mask_id, seed
        self.cls, self.sep = tok.token_to_id("[CLS]"), tok.token_to_id("[SEP]")
        self.store = [self.new_batch()]
        self.n_records = 0

    def new_batch(self):
        B, S = self.B, self.S
        return {"input_ids": np.zeros((B, S), np.int32), "attention_mask": np.ones((B, S), np.int32),
                "token_type_ids": np.zeros((B, S), np.int32), "labels": np.full((B, S), -100, np.int32),
                "index": 0}

    def put(self, b, ids, rec, chunk):
        S, r = self.S, b["index"]
        l = min(S, len(ids))
        b["input_ids"][r, :l] = ids[:l]
        if len(ids) < S:
            b["attention_mask"][r, S - len(ids):] = 0
        keys = mlm_keys(self.seed, rec, chunk, S)
        order = sorted(range(S), key=lambda p: (keys[p], p))
        for p in order[:self.mask_length]:
            if b["input_ids"][r, p] != 0:
                b["labels"][r, p] = b["input_ids"][r, p]
                b["input_ids"][r, p] = self.mask_id
        b["index"] += 1

    def create_sync_batch(self, text):
        rec = self.n_records
        self.n_records += 1
        ids = [self.cls] + self.tok.encode(text, add_special_tokens=True).ids + [self.sep, self.sep]
        if len(ids) < 64:
            return None
        for k, off in enumerate(range(0, len(ids), self.S)):
            self.put(self.store[-1], ids[off:off + self.S], rec, k)
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
    cases = [{"text": t, "ids": tok.encode(t, add_special_tokens=True).ids} for t in recs + edge_cases()]
    with open(os.path.join(HERE, "bert_ids.json"), "w", encoding="utf-8") as f:
        json.dump({"generator": "tokenizers " + __import__("tokenizers").__version__,
                   "asset": "streaming_data_loader_amd/assets/bert_proxy/tokenizer.json",
                   "n_fixture_records": len(recs), "cases": cases}, f, ensure_ascii=False)
    # configs[0]: seq_len=128, batch=8; mask_length = (128 as f32 * 0.15) as usize = 19; mask id 103
    S, B = 128, 8
    pb = PyBatcher(tok, B, S, int(np.float32(S) * np.float32(0.15)), 103, seed=1234)
    out = []
    for t in recs:
        b = pb.create_sync_batch(t)
        if b is not None:
            out.append(b)
    flushed = pb.get_working_batch()
    out.append(flushed)
    arrs = {}
    for i, b in enumerate(out):
        for k in ("input_ids", "attention_mask", "token_type_ids", "labels"):
            arrs[f"b{i}_{k}"] = b[k]
        arrs[f"b{i}_rows"] = np.int32(b["index"])
    arrs["n_batches"] = np.int32(len(out))
    np.savez_compressed(os.path.join(HERE, "mlm_s128_b8.npz"), **arrs)
    print(f"{len(cases)} id cases, {len(out)} mlm batches (last has {out[-1]['index']} rows)", file=sys.stderr)


if __name__ == "__main__":
    main()
