#!/usr/bin/env python3
"""Golden vectors for NFD canonical ordering in the BERT normalizer.

The proxy vocab holds none of the combining marks that survive
strip_accents, so every word carrying them encodes to [UNK] and their order
never shows in the ids.  This script widens the proxy vocab with each kept
mark (and the chars that precomposed symbols decompose to) as a word and as a
"##" continuation, so greedy WordPiece spells such words out char by char and
the ids show the order the normalizer left the marks in.

Writes tests/golden/bert_marks/{tokenizer.json,vocab.txt} and
tests/golden/bert_marks_ids.json (ids from HF `tokenizers`, the project the
reference calls at rust/src/tokenizer/tokenizer_holder.rs:22).  Kept marks and
run separators are found by probing the normalizer itself, the same way
tools/make_unicode_tables.py builds the table the oracle and the device use.
"""
import json
import os
import random
import unicodedata

from tokenizers import Tokenizer
from tokenizers.normalizers import BertNormalizer

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
ASSET = os.path.join(REPO, "streaming_data_loader_amd", "assets", "bert_proxy", "tokenizer.json")
OUT = os.path.join(HERE, "bert_marks")
HI, LO = "\U0001D16D", "\U0001D165"  # ccc 226, ccc 216


def probe():
    norm = BertNormalizer(clean_text=True, handle_chinese_chars=True, strip_accents=None, lowercase=True)
    n = norm.normalize_str
    kept, starter_marks, precomposed, separators, transparent = [], [], [], [], []
    for cp in range(0x80, 0x110000):
        if 0xD800 <= cp <= 0xDFFF:
            continue
        c = chr(cp)
        if unicodedata.combining(c) and n("x" + c) == "x" + c:
            # marks newer than the normalizer's tables are starters to it
            (starter_marks if n("x" + HI + c + LO) == "x" + HI + c + LO else kept).append(c)
    keptset = set(kept)
    for cp in range(0x80, 0x110000):
        if 0xD800 <= cp <= 0xDFFF:
            continue
        c = chr(cp)
        r = n(c)
        if r and r != c and any(ch in keptset for ch in r):
            precomposed.append(c)
        if r == "":
            probe_s = n("x" + HI + c + LO)
            (separators if probe_s == "x" + HI + LO else transparent).append(c)
    return n, kept, starter_marks, precomposed, separators, transparent


def cases(kept, starter_marks, precomposed, separators, transparent):
    out = [
        "x" + HI + LO, "x" + LO + HI, "x" + HI + LO + HI + LO,
        "x\U0001D165᭄", "x᭄\U0001D165", "\U0001D15F᭄", "᭄\U0001D15F",
        "x" + HI + "͏" + LO, "x" + HI + "̀" + LO, "x" + HI + "​" + LO, "x" + HI + "\x00" + LO,
        "x" + HI + " " + LO, "x" + HI + "a" + LO, HI + LO, LO + HI + "x",
        "x" + HI + "́̂" + LO + "y",
    ]
    rng = random.Random(0x0CC)
    starters = list("abcxyz")
    for _ in range(400):
        s = []
        for _ in range(rng.randint(1, 24)):
            r = rng.random()
            if r < 0.45:
                s.append(rng.choice(kept))
            elif r < 0.55:
                s.append(rng.choice(starters))
            elif r < 0.6:
                s.append(rng.choice(starter_marks))
            elif r < 0.7:
                s.append(rng.choice(precomposed))
            elif r < 0.8:
                s.append(rng.choice(separators))
            elif r < 0.9:
                s.append(rng.choice(transparent))
            elif r < 0.95:
                s.append(" ")
            else:
                s.append(rng.choice("!.,中"))
        out.append("".join(s))
    return out


def main():
    n, kept, starter_marks, precomposed, separators, transparent = probe()
    print(f"{len(kept)} kept marks, {len(starter_marks)} marks the normalizer takes as starters, "
          f"{len(precomposed)} precomposed, {len(separators)} separators, "
          f"{len(transparent)} transparent removed chars")
    with open(ASSET, encoding="utf-8") as f:
        tj = json.load(f)
    vocab = tj["model"]["vocab"]
    extra = set(kept) | set(starter_marks)
    for c in precomposed:
        extra.update(n(c))
    for c in sorted(extra):
        for piece in (c, "##" + c):
            if piece not in vocab:
                vocab[piece] = len(vocab)
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, "tokenizer.json"), "w", encoding="utf-8") as f:
        json.dump(tj, f, ensure_ascii=False)
    inv = sorted(vocab.items(), key=lambda kv: kv[1])
    assert [i for _, i in inv] == list(range(len(inv)))
    with open(os.path.join(OUT, "vocab.txt"), "w", encoding="utf-8") as f:
        f.write("".join(k + "\n" for k, _ in inv))
    tok = Tokenizer.from_file(os.path.join(OUT, "tokenizer.json"))
    cs = cases(kept, starter_marks, precomposed, separators, transparent)
    out = {"generator": "tokenizers " + __import__("tokenizers").__version__,
           "asset": "tests/golden/bert_marks/tokenizer.json",
           "cases": [{"text": t, "ids": tok.encode(t, add_special_tokens=True).ids} for t in cs]}
    # the widened vocab must make order visible: a reordered case differs from its naive spelling
    n_reordered = sum(1 for t in cs if n(t) != "".join(n(ch) for ch in t))
    out["n_reordered"] = n_reordered
    print(f"{len(cs)} cases, {n_reordered} where NFD reordering changes the normalized text")
    with open(os.path.join(HERE, "bert_marks_ids.json"), "w", encoding="utf-8") as f:
        json.dump(out, f, ensure_ascii=False, indent=0)


if __name__ == "__main__":
    main()
