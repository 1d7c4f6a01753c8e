#!/usr/bin/env python3
"""A t5 Unigram tokenizer.json that holds the pieces of the reference's t5 known-answer
vector at their real t5-small ids (test infrastructure: the fixture of tests/test_t5_kat.py
and tests/test_gpu_t5_kat.py).

The reference holds one t5 output: `/root/reference/python/test_t5.py:3-7` encodes
"I am here to save the day. The dog is done with the food." with t5-small and records
    [27, 183, 270, 12, 1097, 8, 239, 5, 37, 1782, 19, 612, 28, 8, 542, 5, 1]
(add_special_tokens=True: the `$A </s>` template).  Every word there is one piece (the
last one of "day." / "food." is ".", id 5), so the ids fix these pieces at their indices:
    ▁I 27, ▁am 183, ▁here 270, ▁to 12, ▁save 1097, ▁the 8, ▁day 239, . 5, ▁The 37,
    ▁dog 1782, ▁is 19, ▁done 612, ▁with 28, ▁food 542, </s> 1.

The tokenizer built here is the t5 proxy asset (the real sizes and special-id layout: 32,000
pieces, <pad> </s> <unk> at 0-2, <extra_id_0..99> at 32099..32000, the nmt_nfkc Precompiled
charsmap, WhitespaceSplit + Metaspace, the `$A </s>` template) with those pieces moved to
their t5-small ids: the proxy's own copies of the strings are dropped, and the proxy
pieces that sat at the KAT ids take the freed slots, so the vocabulary stays the proxy's
(realistic competition for every substring) apart from the pinned pieces.  A pinned piece
takes the score of the proxy piece at the same id: sentencepiece numbers pieces by
descending score, so the score at rank i is what a piece at t5-small id i carries in a
vocabulary of this size ("▁am" is no proxy piece; the others keep their place in the score
order).  Nothing is tuned to make the expected split win: the Viterbi has to find it
against the full vocabulary.

Usage: python tests/golden/make_t5_kat_vocab.py [OUT_DIR]  (default tests/golden/t5_kat)
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
TEMPLATE = os.path.join(REPO, "streaming_data_loader_amd", "assets", "t5_proxy", "tokenizer.json")

# /root/reference/python/test_t5.py:3-7
KAT_TEXT = "I am here to save the day. The dog is done with the food."
KAT_IDS = [27, 183, 270, 12, 1097, 8, 239, 5, 37, 1782, 19, 612, 28, 8, 542, 5, 1]
KAT_PIECES = {27: "▁I", 183: "▁am", 270: "▁here", 12: "▁to", 1097: "▁save", 8: "▁the", 239: "▁day", 5: ".",
              37: "▁The", 1782: "▁dog", 19: "▁is", 612: "▁done", 28: "▁with", 542: "▁food"}


def build(template=TEMPLATE):
    with open(template, encoding="utf-8") as f:
        tok = json.load(f)
    vocab = tok["model"]["vocab"]
    n = len(vocab)
    pinned = set(KAT_PIECES.values())
    out = [None] * n
    for i, p in KAT_PIECES.items():
        out[i] = [p, vocab[i][1]]  # the rank's score
    # the other proxy pieces (not pinned strings), by descending score, fill the free slots
    # in order (special / added-token slots keep their own entries)
    reserved = {i for i in range(n) if vocab[i][0].startswith("<") and vocab[i][0].endswith(">") and
                (i < 3 or i >= 32000)}
    for i in reserved:
        out[i] = list(vocab[i])
    rest = [e for i, e in enumerate(vocab) if i not in reserved and e[0] not in pinned]
    rest = sorted(rest, key=lambda e: -e[1])  # (stable: keep the proxy's order among equal scores)
    free = [i for i in range(n) if out[i] is None]
    # "▁am" is new: the proxy's lowest-scored piece gives up its slot (the size stays 32,100)
    rest = rest[:len(free)]
    assert len(rest) == len(free), (len(rest), len(free))
    for i, e in zip(free, rest):
        out[i] = list(e)
    assert len({p for p, _ in out}) == n  # no duplicate strings
    tok["model"]["vocab"] = out
    return tok


def main():
    out_dir = sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "t5_kat")
    os.makedirs(out_dir, exist_ok=True)
    tok = build()
    path = os.path.join(out_dir, "tokenizer.json")
    with open(path, "w", encoding="utf-8") as f:
        json.dump(tok, f, ensure_ascii=False)
    print(path)


if __name__ == "__main__":
    main()
