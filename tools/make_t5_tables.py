#!/usr/bin/env python3
"""Per-code-point tables for the t5 (Precompiled + Unigram) tokenizer path.

The hub t5-small tokenizer.json normalizes with `Precompiled` (crate
tokenizers 0.13.1, normalizers/precompiled.rs): the text is cut into
*extended grapheme clusters* (crate unicode-segmentation, UAX #29) and each
cluster shorter than 6 bytes is looked up whole in the sentencepiece charsmap
trie before falling back to one lookup per char.  The cluster boundaries need
the Grapheme_Cluster_Break, Extended_Pictographic and Indic_Conjunct_Break
properties of every code point; WhitespaceSplit needs White_Space
(char::is_whitespace).  This script writes them, one byte per code point, as
a two-level table:

    "SDLU" u32 version=1 u32 n_pages(=0x110000/256) u32 n_blocks
    u16 page[n_pages]      block index of each 256-code-point page
    u8  block[n_blocks][256]
        bits 0-3  GCB: 0 Other 1 CR 2 LF 3 Control 4 Extend 5 ZWJ 6 RI
                       7 Prepend 8 SpacingMark 9 L 10 V 11 T 12 LV 13 LVT
        bit  4    Extended_Pictographic
        bits 5-6  InCB: 0 None 1 Linker 2 Consonant 3 Extend
        bit  7    White_Space

Properties come from the `regex` module's Unicode data (the same UAX #29
rules it applies for \\X, which tests/test_t5_oracle.py checks the oracle's
segmentation against).  Also prints facts about the proxy charsmap's keys
that the GPU kernel relies on (no key starts with U+0020 or a Prepend char).

Output (committed): streaming_data_loader_amd/data/t5_graphemes.bin
"""
import base64
import json
import os
import struct
import sys

import regex

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "streaming_data_loader_amd", "data", "t5_graphemes.bin")
TOK = os.path.join(REPO, "streaming_data_loader_amd", "assets", "t5_proxy", "tokenizer.json")

GCB = ["Other", "CR", "LF", "Control", "Extend", "ZWJ", "Regional_Indicator", "Prepend", "SpacingMark",
       "L", "V", "T", "LV", "LVT"]
INCB = {"Linker": 1, "Consonant": 2, "Extend": 3}
# char::is_whitespace == the White_Space property
WHITE_SPACE = [0x09, 0x0A, 0x0B, 0x0C, 0x0D, 0x20, 0x85, 0xA0, 0x1680] + list(range(0x2000, 0x200B)) + \
    [0x2028, 0x2029, 0x202F, 0x205F, 0x3000]


def props():
    cps = [c for c in range(0x110000) if not 0xD800 <= c <= 0xDFFF]
    s = "".join(map(chr, cps))
    val = bytearray(0x110000)

    def mark(pattern, setter):
        for m in regex.finditer(pattern + "+", s):
            for i in range(m.start(), m.end()):
                setter(cps[i])

    for k, name in enumerate(GCB):
        if k == 0:
            continue
        def st(c, k=k):
            val[c] = (val[c] & 0xF0) | k
        mark(r"\p{Grapheme_Cluster_Break=%s}" % name, st)
    def ep(c):
        val[c] |= 0x10
    mark(r"\p{Extended_Pictographic}", ep)
    for name, k in INCB.items():
        def st2(c, k=k):
            val[c] = (val[c] & ~0x60) | (k << 5)
        mark(r"\p{Indic_Conjunct_Break=%s}" % name, st2)
    for c in WHITE_SPACE:
        val[c] |= 0x80
    # surrogates: Control (never reach the tokenizer; a Rust String holds none)
    for c in range(0xD800, 0xE000):
        val[c] = 3
    return val


def write_table(val):
    pages, blocks, index = [], [], {}
    for p in range(0x110000 // 256):
        blk = bytes(val[p * 256:(p + 1) * 256])
        if blk not in index:
            index[blk] = len(blocks)
            blocks.append(blk)
        pages.append(index[blk])
    with open(OUT, "wb") as f:
        f.write(b"SDLU" + struct.pack("<III", 1, len(pages), len(blocks)))
        f.write(struct.pack("<%dH" % len(pages), *pages))
        for b in blocks:
            f.write(b)
    print(f"wrote {OUT}: {len(blocks)} blocks", file=sys.stderr)


def charsmap_keys(cm):
    """All (key bytes, normalized str) of a sentencepiece precompiled charsmap."""
    (tsize,) = struct.unpack_from("<I", cm, 0)
    units = struct.unpack_from("<%dI" % (tsize // 4), cm, 4)
    blob = cm[4 + tsize:]

    def offset(u):
        return (u >> 10) << ((u & (1 << 9)) >> 6)

    out = []

    def dfs(pos, key):
        for c in range(1, 256):
            p = pos ^ c
            if p >= len(units) or (units[p] & ((1 << 31) | 0xFF)) != c:
                continue
            q = p ^ offset(units[p])
            k2 = key + bytes([c])
            if (units[p] >> 8) & 1:
                v = units[q] & ((1 << 31) - 1)
                e = blob.index(b"\0", v)
                out.append((k2, blob[v:e].decode("utf-8")))
            dfs(q, k2)

    dfs(offset(units[0]), b"")
    return out


def analyse(val):
    with open(TOK, encoding="utf-8") as f:
        tj = json.load(f)
    cm = base64.b64decode(tj["normalizer"]["precompiled_charsmap"])
    keys = charsmap_keys(cm)
    first = [k.decode("utf-8", "replace")[0] for k, _ in keys]
    sp = [k for k, _ in keys if k[0] == 0x20]
    prep = [k for k, f in zip(keys, first) if (val[ord(f)] & 15) == 7]
    multi = [k for k, _ in keys if len(k.decode("utf-8", "replace")) > 1]
    print(f"charsmap: {len(cm)} bytes, {len(keys)} keys, max key {max(len(k) for k, _ in keys)} bytes, "
          f"max value {max(len(v.encode()) for _, v in keys)} bytes; keys starting with ' ': {len(sp)}; "
          f"starting with a Prepend char: {len(prep)}; multi-char keys: {len(multi)}", file=sys.stderr)
    assert not sp and not prep
    return keys


if __name__ == "__main__":
    v = props()
    write_table(v)
    if os.path.exists(TOK):
        analyse(v)
