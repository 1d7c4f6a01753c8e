#!/usr/bin/env python3
"""Probe the GPT-2 ByteLevel pre-tokenizer regex classes per code point.

The ByteLevel pre-tokenizer of HF `tokenizers` (crate 0.13.1 in the reference,
rust/Cargo.lock; onig 6.4.0) splits with
    's|'t|'re|'ve|'m|'ll|'d| ?\\p{L}+| ?\\p{N}+| ?[^\\s\\p{L}\\p{N}]+|\\s+(?!\\S)|\\s+
so each code point falls in exactly one of four classes: L (\\p{L}), N
(\\p{N}), W (\\s) or O (everything else).  The class is probed from the
installed binding (0.22.2) by pre-tokenizing "a"+c, "1"+c and "!"+c: c joins the
piece of its left neighbour iff it is in that neighbour's class.

Output (committed): streaming_data_loader_amd/data/gpt2_classes.bin
  "SDLG" u32 version=1, u32 n_pages (=4352 pages of 256 code points),
  u32 n_blocks, u16 page_to_block[n_pages], then n_blocks x 64-byte blocks of
  2-bit classes (0=O 1=L 2=N 3=W), code point k of a page at bits 2*(k%4) of byte k/4.
"""
import os
import struct
import sys

from tokenizers import pre_tokenizers

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "streaming_data_loader_amd", "data", "gpt2_classes.bin")
O, L, N, W = 0, 1, 2, 3


def main():
    pt = pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=True)
    cls = bytearray(0x110000)
    counts = [0, 0, 0, 0]
    for cp in range(0x110000):
        if 0xD800 <= cp <= 0xDFFF:
            cls[cp] = O  # not encodable in UTF-8 text; never reached
            continue
        c = chr(cp)
        got = []
        for left, k in (("a", L), ("1", N), ("!", O)):
            if len(pt.pre_tokenize_str(left + c)) == 1:
                got.append(k)
        if c == "'":
            got = [O]  # "!'" is one O-run; contractions are handled by rule
        if len(got) > 1:
            raise SystemExit(f"U+{cp:04X} in several classes {got}")
        k = got[0] if got else W
        if k == W:  # confirm: a whitespace char never joins a letter run
            assert len(pt.pre_tokenize_str("a" + c + "a")) >= 2, hex(cp)
        cls[cp] = k
        counts[k] += 1
    pages, blocks, index = [], [], {}
    for p in range(0x110000 // 256):
        blk = bytearray(64)
        for k in range(256):
            blk[k >> 2] |= cls[p * 256 + k] << (2 * (k & 3))
        b = bytes(blk)
        if b not in index:
            index[b] = len(blocks)
            blocks.append(b)
        pages.append(index[b])
    with open(OUT, "wb") as f:
        f.write(b"SDLG" + struct.pack("<III", 1, len(pages), len(blocks)))
        f.write(struct.pack(f"<{len(pages)}H", *pages))
        for b in blocks:
            f.write(b)
    print(f"O={counts[O]} L={counts[L]} N={counts[N]} W={counts[W]} pages={len(pages)} blocks={len(blocks)}",
          file=sys.stderr)
    print("ascii W:", [hex(c) for c in range(128) if cls[c] == W], file=sys.stderr)


if __name__ == "__main__":
    main()
