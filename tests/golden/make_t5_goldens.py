#!/usr/bin/env python3
"""Generate the t5 (Precompiled + Unigram) golden vectors under tests/golden/.

  t5_ids.json       Tokenizer.encode(text, add_special_tokens=True).ids with the
                    proxy t5-small asset (tools/make_proxy_t5.py) from the HF
                    `tokenizers` binding (0.22.2 here; the reference pins the
                    same project's crate at 0.13.1 and calls it at
                    rust/src/tokenizer/tokenizer_holder.rs:22), for the fixture
                    records, normalizer/grapheme/Unigram edge cases and seeded
                    random strings; plus the Precompiled normalizer output and
                    the `regex` module's \\X cluster starts of each string.
  span_s128_b8.npz  every batch GenTokenizer + T5Data (Span 16.0/2.0) emits on
                    the fixture stream at seq_len=128, batch=8, then the
                    end-of-stream flush (gen_batcher.rs:69-98,
                    t5_data.rs:162-226), under the RNG contract,
                    from the pure-Python restatement below;
  span_rand_s128_b8.npz  the same in rng_mode 1: each row's gap / size draws are
                    rand_distr StandardNormal samples of StdRng::from_seed(seed |
                    record | chunk) (randref.py, pinned by rand_distr's
                    value-stability vector).

Run in the build container:  python tests/golden/make_t5_goldens.py
"""
import json
import math
import os
import random
import sys

import numpy as np
import regex
from tokenizers import Tokenizer

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
ASSET = os.path.join(REPO, "streaming_data_loader_amd", "assets", "t5_proxy", "tokenizer.json")
sys.path.insert(0, HERE)
from make_goldens import philox4x32_10, records  # noqa: E402
from randref import StdRng, row_seed, sat_usize, std_normal  # noqa: E402

M32 = 0xFFFFFFFF


def edge_cases():
    return [
        "", " ", "\t\n\r", "\x00", "a\x00b", "\x0b", "a\x0bb", "a\x01b", "x\x7fy", "\x1c\x1d\x1e\x1f",
        "▁", "a▁b", "▁▁x", "x▁", "  a  b  ", " x　y​z﻿w\u0085v", "a\r\nb", "a\ŕ",
        "</s>", "<pad>x</s>y", "<extra_id_0>", "<extra_id_99>", "<extra_id_100>", "<extra_id_1><extra_id_10>",
        "a<unk>b", "<<pad>>", "<extra_id_5", "x</s></s>", "</s",
        "ＡＢＣ ｆｕｌｌ", "＜unk＞ ＜extra_id_3＞ ＜/s＞", "ﬁne ﬂow", "㎏ ㎞ ① ™ ½ ¼ ℃", "Ⅻ ⅻ",
        "Ầ", "Ầ̀̀", "é", "é́", " ́x",
        " ́x", "\t́x", "x́̂̃̄", "̀́", "́", "Å Å Å",
        "한국어 텍스트", "각 가", "👩‍👩‍👧 👍🏽", "🇩🇪🇫🇷🇩", "😀😀 😀a😀",
        "क्षत्रिय ক্ষ", "؀ x", "a؀b", "؀؀ ́",
        "café naïve résumé Zürich", "İstanbul ß ẞ", "中文字符 日本語 かな カナ", "Ελληνικά русский",
        "a" * 300, "x" * 17 + " " + "y" * 40, "https://en.wikipedia.org/wiki/Foo_(bar)?a=1&b=2",
        "1234567890" * 8, "---===***", "don't won't y'all", "e.g. i.e. U.S.A.",
    ]


def random_strings(n, seed=23):
    rng = random.Random(seed)
    alpha = list("abcdefghijklmnopqrstuvwxyz ABCXYZ     \n\n\t'.,;:!?-()0123456789") + \
        ["é", "é", "́", "̂", "ß", "İ", "Ａ", "ｘ", "ﬁ", "㎏", "中", "😀", "‍", "🇩", "🇪",
         " ", "　", "​", "▁", "<extra_id_7>", "</s>", "<pad>", "\r\n", "\x00", "\x0b", "\x01",
         "한", "ᄀ", "ᅡ", "ᆨ", "क", "्", "ष", "؀", "ः", "ৌ"]
    return ["".join(rng.choice(alpha) for _ in range(rng.randint(0, 50))) for _ in range(n)]


def span_table(avg, lo, cap=32):
    """orc_span_table: thr[j] = floor(2^32 P(trunc_sat(avg - z) <= kmin + j))."""
    k0 = math.floor(avg - 10.0)
    k0 = max(k0, lo)
    thr = []
    for j in range(cap):
        cdf = 0.5 * math.erfc((avg - (k0 + j) - 1.0) / math.sqrt(2.0))
        t = math.floor(cdf * 4294967296.0)
        if t >= 4294967296:
            break
        thr.append(t)
    return k0, thr


def span_pick(tab, x):
    k0, thr = tab
    return k0 + sum(1 for t in thr if t <= x)


class PySpan:
    """GenTokenizer(chunk=true) + T5Data (Span) restated in Python."""

    def __init__(self, tok, B, S, seed, gap=16.0, size=2.0, rng_mode=0):
        self.tok, self.B, self.S, self.seed = tok, B, S, seed
        self.rng_mode, self.avg_gap, self.avg_size = rng_mode, gap, size
        self.eos = tok.token_to_id("</s>")
        self.extra = [tok.token_to_id(f"<extra_id_{k}>") for k in range(100)]
        self.gap, self.size = span_table(gap, 0), span_table(size, 1)
        self.store = [self.new_batch()]
        self.rec = 0
        self.errors = 0

    def new_batch(self):
        B, S = self.B, self.S
        return {"input_ids": np.zeros((B, S), np.int32), "attention_mask": np.ones((B, S), np.int32),
                "labels": np.full((B, S // 4), -100, np.int32), "index": 0}

    def put(self, b, ids, rec, chunk):
        S, r, n = self.S, b["index"], len(ids)
        inp, lab = b["input_ids"][r], b["labels"][r]

        def setlab(i, v):
            if i < S // 4:
                lab[i] = v
            else:
                self.errors += 1

        ip = lp = ap = 0
        p = 0
        rng = StdRng(row_seed(self.seed, rec, chunk)) if self.rng_mode == 1 else None
        while lp < S:
            if rng is None:
                xg, xs = philox4x32_10([p, chunk | 0x40000000, rec & M32, rec >> 32], self.seed & M32, self.seed >> 32)[:2]
                g = span_pick(self.gap, xg)
            else:  # rng_mode 1: random_data_gap / random_data_size on the row's StdRng (t5_data.rs:165-176)
                g = sat_usize(self.avg_gap - std_normal(rng))
            g = min(g, S - lp, n - ip)
            inp[lp:lp + g] = ids[ip:ip + g]
            lp += g
            ip += g
            s = span_pick(self.size, xs) if rng is None else max(sat_usize(self.avg_size - std_normal(rng)), 1)
            s = min(s, S - lp, n - ip)
            if s > 0:
                inp[lp] = self.extra[p]
                setlab(ap, self.extra[p])
                for i in range(s):
                    setlab(ap + i + 1, ids[ip + i])
                lp += 1
                ip += s
                ap += s + 1
            if n <= ip:
                setlab(ap, self.extra[p + 1])
                break
            p += 1
        b["index"] += 1

    def create_sync_batch(self, text):
        rec = self.rec
        self.rec += 1
        ids = [self.eos] + self.tok.encode(text, add_special_tokens=True).ids + [self.eos]
        if len(ids) < 64:
            return None
        for c, off in enumerate(range(0, len(ids), self.S)):
            self.put(self.store[-1], ids[off:off + self.S], rec, c)
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
    cases = []
    for t in recs + edge_cases() + random_strings(400):
        cases.append({"text": t, "ids": tok.encode(t, add_special_tokens=True).ids,
                      "norm": tok.normalizer.normalize_str(t),
                      "graphemes": [m.start() for m in regex.finditer(r"\X", t)]})
    with open(os.path.join(HERE, "t5_ids.json"), "w", encoding="utf-8") as f:
        json.dump({"generator": "tokenizers " + __import__("tokenizers").__version__ + ", regex " + regex.__version__,
                   "asset": "streaming_data_loader_amd/assets/t5_proxy/tokenizer.json",
                   "n_fixture_records": len(recs), "cases": cases}, f, ensure_ascii=False)
    for mode, name in ((0, "span_s128_b8.npz"), (1, "span_rand_s128_b8.npz")):
        write_span_batches(tok, recs, mode, name)


def write_span_batches(tok, recs, rng_mode, name):
    ps = PySpan(tok, 8, 128, seed=1234, rng_mode=rng_mode)
    out = [b for b in (ps.create_sync_batch(t) for t in recs) if b is not None]
    out.append(ps.get_working_batch())
    arrs = {}
    for i, b in enumerate(out):
        for k in ("input_ids", "attention_mask", "labels"):
            arrs[f"b{i}_{k}"] = b[k]
        arrs[f"b{i}_rows"] = np.int32(b["index"])
    arrs["n_batches"] = np.int32(len(out))
    arrs["span_errors"] = np.int64(ps.errors)
    arrs["gap_table"] = np.array([ps.gap[0]] + ps.gap[1], np.int64)
    arrs["size_table"] = np.array([ps.size[0]] + ps.size[1], np.int64)
    np.savez_compressed(os.path.join(HERE, name), **arrs)
    print(f"{name}: {len(out)} span batches (last has {out[-1]['index']} rows), "
          f"{ps.errors} label overflows", file=sys.stderr)


if __name__ == "__main__":
    main()
