"""Pins the CPU oracle on diverse text against `tokenizers` itself
(tests/golden/make_heldout_goldens.py, tokenizers 0.22.2; the reference pins
the same project's crate at 0.13.1 and calls it at
rust/src/tokenizer/tokenizer_holder.rs:22):

- the 523 held-out records (3.0 MB; text the proxy vocabularies were not
  trained on) through all three proxy tokenizers, compared per record by id
  count and blake2b-64 digest of the ids;
- 3000 seeded random-Unicode and long-identifier strings, id for id;
- JSON number parsing: the f64 tokenizers holds for a Unigram score is
  serde_json's default two-rounding parse, not the correctly rounded value
  (an ulp apart for ~1/4 of 17-digit scores), and that decides Viterbi ties:
  a held-out record whose "=" run splits into equal-sum piece sequences.
"""
import hashlib
import json
import os
import struct

import numpy as np
import pytest

import oracle_lib

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def g():
    return np.load(os.path.join(GOLDEN, "heldout_ids.npz"))


def digest_ids(ids):
    return int.from_bytes(hashlib.blake2b(np.asarray(ids, "<u4").tobytes(), digest_size=8).digest(), "little")


def heldout_records():
    with open(os.path.join(GOLDEN, "heldout_records.jsonl"), encoding="utf-8") as f:
        return [json.loads(l)["text"] for l in f]


def generated(g):
    t, o = g["gen_text"], g["gen_off"]
    return [t[o[i]:o[i + 1]].tobytes() for i in range(len(o) - 1)]


def oracle_encoder(kind):
    return {"bert": oracle_lib.Tok, "gpt2": oracle_lib.Gpt2Tok, "t5": oracle_lib.T5Tok}[kind]()


def test_serde_numbers_match_tokenizers(g):
    t, o, want = g["serde_text"], g["serde_off"], g["serde_f64"]
    assert len(want) > 1000
    bad = []
    for i in range(len(want)):
        s = t[o[i]:o[i + 1]].tobytes()
        got = struct.unpack("<Q", struct.pack("<d", oracle_lib.json_number(s)))[0]
        if got != int(want[i]):
            bad.append(s.decode())
    assert not bad, f"{len(bad)} numbers differ, e.g. {bad[:5]}"
    # the parse is not strtod: the first of these lands an ulp from the correctly rounded value
    assert oracle_lib.json_number("-10.234719276428223") != -10.234719276428223
    assert oracle_lib.json_number("-9.60637092590332") == -9.60637092590332


@pytest.mark.parametrize("kind", ["bert", "gpt2", "t5"])
def test_oracle_heldout_corpus_matches_tokenizers(g, kind):
    recs = heldout_records()
    assert len(recs) == len(g[f"{kind}_n"]) == 523
    tok = oracle_encoder(kind)
    bad = []
    for i, r in enumerate(recs):
        ids = tok.encode(r)
        if len(ids) != int(g[f"{kind}_n"][i]) or digest_ids(ids) != int(g[f"{kind}_digest"][i]):
            bad.append(i)
    assert not bad, f"{len(bad)} of {len(recs)} records differ, first {bad[:5]}"


@pytest.mark.parametrize("kind", ["bert", "gpt2", "t5"])
def test_oracle_generated_strings_match_tokenizers(g, kind):
    texts = generated(g)
    assert len(texts) == 3000
    ids, off = g[f"{kind}_ids"], g[f"{kind}_off"]
    tok = oracle_encoder(kind)
    bad = [i for i, b in enumerate(texts) if tok.encode(b) != ids[off[i]:off[i + 1]].tolist()]
    assert not bad, f"{len(bad)} of {len(texts)} strings differ, e.g. {[texts[i][:40] for i in bad[:3]]}"
