#!/usr/bin/env python3
"""Derive the per-codepoint BertNormalizer + BertPreTokenizer tables.

The reference's tokenizer arithmetic lives in the third-party crate
`tokenizers 0.13.1` (`rust/Cargo.lock`), not vendored.  Its BertNormalizer
(clean_text, handle_chinese_chars, strip_accents=None->lowercase, lowercase)
and BertPreTokenizer are context-free per codepoint except for the NFD
canonical re-ordering of combining marks that strip_accents keeps, so they are
captured here as tables by probing EVERY codepoint through the same project's
Python binding (`tokenizers 0.22.2`, the version importable in this container):

  N(c)  = BertNormalizer(lowercase=True).normalize_str(chr(c))
  class = how BertPreTokenizer treats N(c):
          DEL   N(c) == ""                (clean_text removals, lone Mn marks)
          WS    N(c) is only whitespace   (split + removed)
          ISO   N(c) is one isolated char (punctuation, or a CJK char padded
                with spaces by handle_chinese_chars) -> a one-char word
          OTHER word character; its normalized bytes are N(c)

Binary layout (little endian), read by oracle/ and by the HIP library:
  char[4] "SDLU", u32 version=2, u32 n_pages, u32 n_blocks, u32 pool_bytes
  u16 page[n_pages]                  block index for codepoints [p*128, p*128+128)
  u32 entry[n_blocks*128]            bits 0-1 class (0 OTHER,1 WS,2 ISO,3 DEL)
                                     bit 2   identity (N(c) == chr(c))
                                     bit 4   canonical ordering (NFD) flag, below
                                     bits 8-31 pool offset of N(c) (if not identity)
  u8  pool[pool_bytes]               at each offset: u8 nbytes, u8 nchars, bytes

Canonical ordering (version 2, bit 4).  NFD sorts every run of combining marks
(ccc > 0) by ccc before strip_accents drops the Mn ones, so the marks it KEEPS
come out of a run in ccc order.  Probed the same way (N("x" + M226 + c + M216)):
  - a kept mark (identity, ccc > 0): bit 4, ccc in bits 8-15;
  - a char whose N(c) contains a kept mark (a precomposed char): bit 4;
  - a DEL char that still ends a run (a removed starter, e.g. an Mn with ccc 0):
    bit 4; other DEL chars (clean_text removals, Mn with ccc > 0) do not.
Everything else either holds a starter (ends the run) or is removed.
"""
import os
import struct
import sys
import unicodedata

from tokenizers import normalizers, pre_tokenizers

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "streaming_data_loader_amd", "data", "bert_uncased_unicode.bin")

OTHER, WS, ISO, DEL = 0, 1, 2, 3


def main():
    norm = normalizers.BertNormalizer(lowercase=True)
    pre = pre_tokenizers.BertPreTokenizer()
    char_kind = {}

    def kind(d):
        k = char_kind.get(d)
        if k is None:
            parts = [p for p, _ in pre.pre_tokenize_str("a" + d + "a")]
            if parts == ["a", "a"]:
                k = WS
            elif parts == ["a", d, "a"]:
                k = ISO
            elif parts == ["a" + d + "a"]:
                k = OTHER
            else:
                raise RuntimeError(f"unexpected pre-tokenization of U+{ord(d):04X}: {parts}")
            char_kind[d] = k
        return k

    entries = [0] * 0x110000
    pool = bytearray()
    pool_index = {}
    mixed = []
    for cp in range(0x110000):
        if 0xD800 <= cp <= 0xDFFF:
            entries[cp] = DEL  # surrogates never occur in valid UTF-8
            continue
        c = chr(cp)
        n = norm.normalize_str(c)
        if n == "":
            entries[cp] = DEL
            continue
        kinds = [kind(d) for d in n]
        core = [d for d, k in zip(n, kinds) if k != WS]
        core_k = [k for k in kinds if k != WS]
        if not core:
            cls = WS
        elif len(core) == 1 and core_k[0] == ISO:
            cls = ISO                       # punctuation: isolated one-char word
        elif len(core) == 1 and len(n) > 1 and all(k == WS for k in kinds if k != OTHER):
            cls = ISO                       # CJK char padded " c " by handle_chinese_chars
        elif all(k == OTHER for k in kinds):
            cls = OTHER                     # word char (possibly several normalized chars)
        else:
            mixed.append((cp, n, kinds))
            cls = OTHER
        mapped = "".join(core)
        e = cls
        if mapped == c:
            e |= 4
        else:
            b = mapped.encode("utf-8")
            key = (b, len(mapped))
            off = pool_index.get(key)
            if off is None:
                off = len(pool)
                pool_index[key] = off
                pool += bytes([len(b), len(mapped)]) + b
            e |= off << 8
        entries[cp] = e
    if mixed:
        print("mixed-class codepoints (handled as OTHER):", len(mixed), mixed[:10], file=sys.stderr)

    # canonical ordering flags (bit 4), probed: H (ccc 226) and L (ccc 216) are kept marks
    H, L = "\U0001D16D", "\U0001D165"
    kept_ccc = {}
    for cp in range(0x110000):
        if 0xD800 <= cp <= 0xDFFF:
            continue
        c = chr(cp)
        n = norm.normalize_str(c)
        r = norm.normalize_str("x" + H + c + L)
        if n == "":
            if r == "x" + H + L:
                entries[cp] |= 16  # a removed starter: ends the run
            elif r != "x" + L + H:
                raise RuntimeError(f"U+{cp:04X}: unexpected ordering {r!r}")
            continue
        if r == "x" + H + n + L:
            continue  # holds a starter
        ccc = unicodedata.combining(c)
        if n != c or ccc == 0:
            raise RuntimeError(f"U+{cp:04X}: reorders but is not a known kept mark")
        want = "x" + "".join(m for _, m in sorted([(226, H), (ccc, c), (216, L)], key=lambda t: t[0]))
        if r != want:
            raise RuntimeError(f"U+{cp:04X}: ccc {ccc} does not explain {r!r}")
        kept_ccc[cp] = ccc
        entries[cp] = (entries[cp] & ~0xFFFFFF00) | 16 | (ccc << 8)
    for cp in range(0x110000):
        e = entries[cp]
        if (e & 3) == OTHER and not (e & 4) and any(ord(x) in kept_ccc for x in norm.normalize_str(chr(cp))):
            entries[cp] |= 16  # precomposed: its decomposition holds kept marks
    print(f"canonical ordering: {len(kept_ccc)} kept marks, "
          f"{sum(1 for e in entries if (e & 3) == DEL and e & 16)} removed starters, "
          f"{sum(1 for cp, e in enumerate(entries) if (e & 3) == OTHER and e & 16 and cp not in kept_ccc)} "
          f"precomposed", file=sys.stderr)

    pages, blocks, block_index = [], [], {}
    for p in range(0x110000 // 128):
        blk = tuple(entries[p * 128:(p + 1) * 128])
        bi = block_index.get(blk)
        if bi is None:
            bi = len(blocks)
            block_index[blk] = bi
            blocks.append(blk)
        pages.append(bi)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "wb") as f:
        f.write(b"SDLU" + struct.pack("<IIII", 2, len(pages), len(blocks), len(pool)))
        f.write(struct.pack(f"<{len(pages)}H", *pages))
        for blk in blocks:
            f.write(struct.pack("<128I", *blk))
        f.write(bytes(pool))
    print(f"pages={len(pages)} blocks={len(blocks)} pool={len(pool)} -> {OUT}", file=sys.stderr)


if __name__ == "__main__":
    main()
