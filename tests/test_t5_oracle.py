"""Pins the t5 CPU oracle (oracle/orc_unigram.c + the span batcher in
oracle/orc_batcher.c) before it is trusted as the checker for task=span.

- token ids, Precompiled normalizer output and grapheme cluster starts against
  HF `tokenizers` 0.22.2 / the `regex` module's \\X on the fixture records,
  edge cases and seeded random strings -- tests/golden/t5_ids.json
  (tests/golden/make_t5_goldens.py);
- span batches at S=128 B=8 against the independent Python restatement of
  GenTokenizer + T5Data under the RNG contract -- tests/golden/span_s128_b8.npz;
- the span draw tables against the same restatement's (math.erfc).
"""
import json
import os
import random

import numpy as np
import pytest

import oracle_lib

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def t5tok():
    return oracle_lib.T5Tok()


@pytest.fixture(scope="module")
def t5_goldens():
    with open(os.path.join(GOLDEN, "t5_ids.json"), encoding="utf-8") as f:
        return json.load(f)


def test_t5_ids_match_tokenizers(t5tok, t5_goldens):
    assert t5_goldens["n_fixture_records"] == 50
    bad = [(c["text"][:40], c["ids"][:12], t5tok.encode(c["text"])[:12]) for c in t5_goldens["cases"]
           if t5tok.encode(c["text"]) != c["ids"]]
    assert not bad, f"{len(bad)} of {len(t5_goldens['cases'])} mismatch, e.g. {bad[:3]}"


def test_t5_normalizer_matches_precompiled(t5tok, t5_goldens):
    bad = [repr(c["text"][:30]) for c in t5_goldens["cases"] if t5tok.normalize(c["text"]) != c["norm"]]
    assert not bad, f"{len(bad)} mismatches, e.g. {bad[:5]}"


def _char_to_byte(text):
    out, b = [], 0
    for ch in text:
        out.append(b)
        b += len(ch.encode("utf-8"))
    return out


def test_t5_graphemes_match_regex(t5tok, t5_goldens):
    bad = []
    for c in t5_goldens["cases"]:
        t = c["text"]
        cb = _char_to_byte(t)
        want = [cb[i] for i in c["graphemes"]]
        if t5tok.grapheme_starts(t) != want:
            bad.append(repr(t[:30]))
    assert not bad, f"{len(bad)} mismatches, e.g. {bad[:5]}"


def test_t5_layout(t5tok):
    assert t5tok.eos == 1
    assert t5tok.special_id("<extra_id_0>") == 32099 and t5tok.special_id("<extra_id_99>") == 32000
    assert t5tok.encode("") == [1]
    assert t5tok.encode("</s>") == [1, 1]
    assert t5tok.encode("<extra_id_0><pad>") == [32099, 0, 1]


def test_span_tables_match_restatement():
    import sys
    sys.path.insert(0, GOLDEN)
    from make_t5_goldens import span_table
    for avg, lo in ((16.0, 0), (2.0, 1), (3.0, 1), (0.5, 0), (100.25, 0)):
        k0, thr = span_table(avg, lo)
        assert oracle_lib.span_table(avg, lo) == (k0, thr), (avg, lo)
    g = np.load(os.path.join(GOLDEN, "span_s128_b8.npz"))
    assert oracle_lib.span_table(16.0, 0) == (int(g["gap_table"][0]), g["gap_table"][1:].tolist())
    assert oracle_lib.span_table(2.0, 1) == (int(g["size_table"][0]), g["size_table"][1:].tolist())


def test_span_table_distribution():
    """The table samples trunc_sat(avg - z), z ~ N(0,1): check its mean."""
    from math import erf, sqrt
    for avg, lo in ((16.0, 0), (2.0, 1)):
        k0, thr = oracle_lib.span_table(avg, lo)
        edges = [0] + thr + [1 << 32]
        p = np.diff(np.array(edges, np.float64)) / 2.0 ** 32
        vals = np.arange(k0, k0 + len(p))
        mean = float((p * vals).sum())
        # E[max(trunc(avg - z), lo)] by numeric integration
        zs = np.linspace(-12, 12, 2_000_001)
        w = np.exp(-zs ** 2 / 2) / sqrt(2 * np.pi)
        v = np.maximum(np.trunc(np.maximum(avg - zs, 0.0)), lo)
        want = float((w * v).sum() * (zs[1] - zs[0]))
        assert abs(mean - want) < 1e-4, (avg, mean, want)


def test_span_batches_match_golden(t5tok, records):
    g = np.load(os.path.join(GOLDEN, "span_s128_b8.npz"))
    enc = oracle_lib.Encoder("t5", t5tok)
    ob = oracle_lib.OracleBatcherEx(enc, oracle_lib.SPAN, 8, 128, seed=1234)
    got = [r for r in (ob.push(t) for t in records) if r is not None]
    got.append(ob.flush())
    assert len(got) == int(g["n_batches"])
    for i, b in enumerate(got):
        assert b["rows"] == int(g[f"b{i}_rows"])
        for k in ("input_ids", "attention_mask", "labels"):
            np.testing.assert_array_equal(b[k], g[f"b{i}_{k}"], err_msg=f"batch {i} {k}")
    assert ob.span_errors() == int(g["span_errors"])


def test_span_row_invariants(t5tok, records):
    """Every row: inputs are the chunk's ids with each span replaced by its
    sentinel, labels are the sentinels followed by the removed ids and a final
    sentinel -- extra[pass + 1], one past the last span's, or two past when the
    last pass's gap reached the end of the chunk (t5_data.rs:189-221)."""
    enc = oracle_lib.Encoder("t5", t5tok)
    S = 512
    ob = oracle_lib.OracleBatcherEx(enc, oracle_lib.SPAN, 4, S, seed=99)
    extra = {32099 - k: k for k in range(100)}
    rows = 0
    for t in records * 3:
        b = ob.push(t)
        if b is None:
            continue
        for r in range(b["rows"]):
            inp, lab = b["input_ids"][r], b["labels"][r]
            sent_in = [x for x in inp if x in extra]
            assert [extra[x] for x in sent_in] == list(range(len(sent_in)))
            lab = lab[lab != -100]
            sent_lab = [extra[x] for x in lab if x in extra]
            assert sent_lab[:-1] == list(range(len(sent_in)))
            assert sent_lab[-1] in (len(sent_in), len(sent_in) + 1)
            rows += 1
    assert rows > 20
    assert ob.span_errors() == 0


def test_grapheme_table_whitespace_and_ascii_match_kernel_arithmetic():
    """tokenize_unigram.hip tests White_Space and an ASCII char's property byte
    arithmetically (common.hpp uni_white_space / uni_ascii_props) instead of
    loading them; the handle checks the loaded table agrees at creation.  The
    same check here on the committed table, without a GPU."""
    import struct
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "streaming_data_loader_amd",
                        "data", "t5_graphemes.bin")
    raw = open(path, "rb").read()
    assert raw[:4] == b"SDLU"
    _, n_pages, n_blocks = struct.unpack_from("<III", raw, 4)
    pages = np.frombuffer(raw, np.uint16, n_pages, 16)
    blocks = np.frombuffer(raw, np.uint8, n_blocks * 256, 16 + 2 * n_pages).reshape(n_blocks, 256)
    props = blocks[pages].reshape(-1)
    assert props.size == 0x110000
    ws = {0x85, 0xA0, 0x1680, 0x2028, 0x2029, 0x202F, 0x205F, 0x3000} | set(range(0x2000, 0x200B)) | \
        set(range(9, 14)) | {32}
    got = set(np.nonzero(props & 0x80)[0].tolist())
    assert got == ws
    for c in range(128):
        gcb = 1 if c == 13 else 2 if c == 10 else 3 if (c < 32 or c == 127) else 0
        assert int(props[c]) == gcb | (0x80 if c in ws else 0), hex(c)
