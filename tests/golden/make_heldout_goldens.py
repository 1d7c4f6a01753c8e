#!/usr/bin/env python3
"""Token-id goldens for diverse text, for all three proxy tokenizers.

Run in the build container (needs the HF `tokenizers` binding, 0.22.2 here;
the reference pins the same project's crate at 0.13.1 and calls it at
rust/src/tokenizer/tokenizer_holder.rs:22):

    python tests/golden/make_heldout_goldens.py

heldout_ids.npz holds, for kind in bert / gpt2 / t5:
  {kind}_n, {kind}_digest   per record of tests/golden/heldout_records.jsonl
                            (523 records, 3.0 MB: CPython help topics, stdlib
                            docstrings, Perl POD, Debian license texts): the
                            number of ids Tokenizer.encode(text, True) gives and
                            the blake2b-64 digest of those ids as little-endian
                            u32 (digest_ids below), so 2.3 M ids fit in 12 KB;
  {kind}_ids, {kind}_off    the full ids of every generated string (CSR);
  gen_text, gen_off         the generated strings (UTF-8, CSR): seeded random
                            Unicode (code points over every plane and the blocks
                            the normalizers and pre-tokenizers treat specially)
                            and long identifiers / URLs / paths / symbol runs;
  serde_text, serde_off,    JSON number texts and the f64 bits tokenizers holds
  serde_f64                 after parsing them as Unigram scores (serde_json's
                            default two-rounding parse, see oracle/orc_json.c).
"""
import hashlib
import json
import os
import random
import struct
import sys

import numpy as np
from tokenizers import Tokenizer

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
ASSETS = os.path.join(REPO, "streaming_data_loader_amd", "assets")
TOKENIZERS = {"bert": "bert_proxy", "gpt2": "gpt2_proxy", "t5": "t5_proxy"}


def digest_ids(ids):
    return int.from_bytes(hashlib.blake2b(np.asarray(ids, "<u4").tobytes(), digest_size=8).digest(), "little")


def heldout_records():
    with open(os.path.join(HERE, "heldout_records.jsonl"), encoding="utf-8") as f:
        return [json.loads(l)["text"] for l in f]


# code-point pools: (lo, hi) ranges the tokenizers' tables treat specially
BLOCKS = [
    (0x00, 0x1F), (0x7F, 0x9F), (0xA0, 0xFF), (0x100, 0x24F), (0x250, 0x2FF), (0x300, 0x36F), (0x370, 0x3FF),
    (0x400, 0x4FF), (0x530, 0x58F), (0x590, 0x5FF), (0x600, 0x6FF), (0x900, 0x97F), (0x980, 0x9FF), (0xE00, 0xE7F),
    (0x1100, 0x11FF), (0x1680, 0x1680), (0x1AB0, 0x1AFF), (0x1DC0, 0x1DFF), (0x1E00, 0x1EFF), (0x2000, 0x206F),
    (0x2070, 0x209F), (0x20A0, 0x20CF), (0x20D0, 0x20FF), (0x2100, 0x214F), (0x2150, 0x218F), (0x2190, 0x21FF),
    (0x2200, 0x22FF), (0x2460, 0x24FF), (0x2500, 0x257F), (0x2700, 0x27BF), (0x2E80, 0x2FDF), (0x3000, 0x303F),
    (0x3040, 0x30FF), (0x3130, 0x318F), (0x3200, 0x33FF), (0x3400, 0x4DBF), (0x4E00, 0x9FFF), (0xA960, 0xA97F),
    (0xAC00, 0xD7A3), (0xD7B0, 0xD7FF), (0xE000, 0xE0FF), (0xF900, 0xFAFF), (0xFB00, 0xFB4F), (0xFDD0, 0xFDEF),
    (0xFE00, 0xFE0F), (0xFE30, 0xFE4F), (0xFF00, 0xFFEF), (0xFFF0, 0xFFFF), (0x10000, 0x1007F), (0x1D400, 0x1D7FF),
    (0x1D165, 0x1D16D), (0x1F1E6, 0x1F1FF), (0x1F300, 0x1F5FF), (0x1F600, 0x1F64F), (0x1F900, 0x1FAFF),
    (0x1F3FB, 0x1F3FF), (0x20000, 0x2A6DF), (0x2F800, 0x2FA1F), (0x30000, 0x3134F), (0xE0000, 0xE007F),
    (0xE0100, 0xE01EF), (0xF0000, 0xF00FF), (0x10FFF0, 0x10FFFF),
]
SPECIALS = ["[CLS]", "[SEP]", "[MASK]", "[PAD]", "[UNK]", "<|endoftext|>", "</s>", "<pad>", "<unk>", "<extra_id_0>",
            "<extra_id_42>", "<extra_id_99>", "##", "▁", "‍", "﻿", "­", "\r\n", "'s", "'ll", "n't"]


def rand_char(rng):
    r = rng.random()
    if r < 0.35:
        return rng.choice("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789 .,;:'\"!?-()[]{}<>/\\_#@$%&*+=~^`|")
    if r < 0.45:
        return rng.choice(" \t\n\r\x0b\x0c\x00")
    while True:
        if r < 0.92:
            lo, hi = rng.choice(BLOCKS)
            cp = rng.randint(lo, hi)
        else:
            cp = rng.randint(0, 0x10FFFF)
        if not 0xD800 <= cp <= 0xDFFF:
            return chr(cp)


def random_unicode(rng, n):
    out = []
    for _ in range(n):
        parts = []
        for _ in range(rng.randint(0, 24)):
            if rng.random() < 0.06:
                parts.append(rng.choice(SPECIALS))
            elif rng.random() < 0.3:  # a run of one block: words of scripts, stacked marks
                lo, hi = rng.choice(BLOCKS)
                parts.append("".join(chr(c) for c in (rng.randint(lo, hi) for _ in range(rng.randint(1, 12)))
                                     if not 0xD800 <= c <= 0xDFFF))
            else:
                parts.append("".join(rand_char(rng) for _ in range(rng.randint(1, 6))))
        out.append("".join(parts))
    return out


WORDS = ["get", "set", "value", "buffer", "index", "token", "stream", "batch", "http", "json", "parse", "encode",
         "utf8", "x86", "id", "max", "min", "len", "tmp", "config", "loader", "shard", "Mask", "Span", "GPU", "HIP"]


def long_identifiers(rng, n):
    out = []
    for _ in range(n):
        k = rng.randrange(12)
        ws = [rng.choice(WORDS) for _ in range(rng.randint(2, 14))]
        if k == 0:
            s = "_".join(w.lower() for w in ws)
        elif k == 1:
            s = ws[0].lower() + "".join(w.capitalize() for w in ws[1:])
        elif k == 2:
            s = ".".join(ws) + "(" + ", ".join(rng.choice(WORDS) for _ in range(rng.randint(0, 3))) + ")"
        elif k == 3:
            s = "https://" + ".".join(ws[:2]) + ".org/" + "/".join(ws[2:]) + "?q=" + str(rng.randrange(10 ** 9))
        elif k == 4:
            s = "/usr/" + "/".join(ws) + rng.choice([".py", ".rs", ".json.gz", ".h", ""])
        elif k == 5:
            s = "".join(rng.choice("0123456789abcdef") for _ in range(rng.randint(17, 130)))
        elif k == 6:
            s = "".join(rng.choice("ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/") for _ in
                        range(rng.randint(17, 200))) + "=" * rng.randint(0, 2)
        elif k == 7:
            s = rng.choice("=-*#~_.+") * rng.randint(17, 160)
        elif k == 8:
            s = rng.choice("xyzaé") * rng.choice([98, 99, 100, 101, 102]) + rng.choice(["", " end", "s"])
        elif k == 9:
            s = "".join(w.upper() if rng.random() < 0.5 else w for w in ws) + str(rng.randrange(10 ** 6))
        elif k == 10:
            s = "-".join(ws) + "--" + "_".join(ws[::-1])
        else:
            s = "".join(ws) + "".join(rng.choice("áéíóúñçüößøåæ") for _ in range(rng.randint(1, 8))) + "".join(ws)
        sep = rng.choice([" ", "\n", "\t", "  ", ", ", "; ", ""])
        out.append(sep.join([s] + ([rng.choice(WORDS)] if rng.random() < 0.5 else [])))
    return out


def serde_number_cases(rng):
    """JSON number texts covering every branch of serde_json's f64 parse."""
    cases = []
    for _ in range(600):  # sentencepiece-style: f32 scores printed as Python f64 reprs
        f = struct.unpack("<f", struct.pack("<f", -rng.uniform(0.0, 25.0)))[0]
        cases.append(repr(f))
    for _ in range(200):  # random decimals of 1..30 significant digits (u64 overflow past 19-20)
        d = rng.randint(1, 30)
        digits = str(rng.randint(1, 9)) + "".join(rng.choice("0123456789") for _ in range(d - 1))
        p = rng.randint(0, len(digits))
        s = digits[:p] + ("." + digits[p:] if p < len(digits) else "")
        s = s if not s.startswith(".") else "0" + s
        cases.append(("-" if rng.random() < 0.7 else "") + s)
    for _ in range(200):  # exponents
        m = f"{rng.randint(1, 10 ** rng.randint(1, 19))}" + (f".{rng.randint(0, 10 ** 6)}" if rng.random() < 0.5 else "")
        es = rng.choice(["", "+", "-"])  # (a positive exponent stays finite: overflow is a parse error)
        cases.append(("-" if rng.random() < 0.5 else "") + m + rng.choice("eE") + es +
                     str(rng.randint(0, 340 if es == "-" else 280)))
    cases += ["0", "-0", "0.0", "-0.0", "1e-400", "-1e-400", "0e999999999999", "18446744073709551615",
              "18446744073709551616", "184467440737095516150.5", "1844674407370955161.5", "1844674407370955161.6",
              "123456789012345678901234567890", "0.000000000000000000000000001", "-10.234719276428223",
              "-11.259500503540039", "-9.60637092590332", "2.2250738585072014e-308", "4.9e-324", "1.7976931348623157e308"]
    return cases


def serde_goldens(cases):
    """Parse each number as a Unigram score through tokenizers itself."""
    vocab = [["<unk>", 0.0]] + [[f"p{i}", 0.0] for i in range(len(cases))]
    body = json.dumps({"version": "1.0", "truncation": None, "padding": None, "added_tokens": [], "normalizer": None,
                       "pre_tokenizer": None, "post_processor": None, "decoder": None,
                       "model": {"type": "Unigram", "unk_id": 0, "vocab": vocab, "byte_fallback": False}})
    # splice the raw number texts in place of the placeholder scores
    parts = body.split(", 0.0]")
    assert len(parts) == len(cases) + 2
    out = parts[0] + ", 0.0]"
    for c, p in zip(cases, parts[1:-1]):
        out += p + ", " + c + "]"
    out += parts[-1]
    tk = Tokenizer.from_str(out)
    held = json.loads(tk.to_str())["model"]["vocab"]
    return [struct.unpack("<Q", struct.pack("<d", float(v[1])))[0] for v in held[1:]]


def csr(seqs, dtype):
    off = np.zeros(len(seqs) + 1, np.int64)
    np.cumsum([len(s) for s in seqs], out=off[1:])
    flat = np.concatenate([np.asarray(s, dtype) for s in seqs]) if seqs else np.zeros(0, dtype)
    return flat, off


def main():
    rng = random.Random(0x5D1B03)
    gen = random_unicode(rng, 2000) + long_identifiers(rng, 1000)
    recs = heldout_records()
    arrs = {}
    for kind, d in TOKENIZERS.items():
        tk = Tokenizer.from_file(os.path.join(ASSETS, d, "tokenizer.json"))
        enc = tk.encode_batch(recs, add_special_tokens=True)
        arrs[f"{kind}_n"] = np.array([len(e.ids) for e in enc], np.int64)
        arrs[f"{kind}_digest"] = np.array([digest_ids(e.ids) for e in enc], np.uint64)
        genc = tk.encode_batch(gen, add_special_tokens=True)
        arrs[f"{kind}_ids"], arrs[f"{kind}_off"] = csr([e.ids for e in genc], np.uint32)
        print(f"{kind}: {int(arrs[kind + '_n'].sum())} held-out ids, {len(arrs[kind + '_ids'])} generated ids",
              file=sys.stderr)
    blobs = [g.encode("utf-8") for g in gen]
    arrs["gen_text"], arrs["gen_off"] = csr([np.frombuffer(b, np.uint8) for b in blobs], np.uint8)
    cases = serde_number_cases(rng)
    arrs["serde_text"], arrs["serde_off"] = csr([np.frombuffer(c.encode(), np.uint8) for c in cases], np.uint8)
    arrs["serde_f64"] = np.array(serde_goldens(cases), np.uint64)
    arrs["generator"] = np.array("tokenizers " + __import__("tokenizers").__version__)
    np.savez_compressed(os.path.join(HERE, "heldout_ids.npz"), **arrs)


if __name__ == "__main__":
    main()
