"""Pin against the one output the reference itself produced: `data/test.bin`.

`tests/golden/testbin_rows.json` (made by `tests/golden/make_testbin_vocab.py` from the
reference's `data/test.bin`) holds the dump's 8 x 128 bert-base-uncased ids -- what
`tokenizers` 0.13.1 returned for the first three records of `data/test.json.gz`
(`rust/src/tokenizer/tokenizer_holder.rs:19-28`) -- the three texts as that (older) provider
handed them over, and the pieces the dump determines at their real ids.

The check: a WordPiece vocabulary holding those pieces (fillers elsewhere) reproduces every
non-wildcard id of the dump -- 1,020 of 1,022 positions -- through
  * `tokenizers` 0.22.2 (the reference's engine, here only the checker of the fixture),
  * the C oracle (`oracle/sdl_oracle.c`), and
  * the HIP path (`tests/test_gpu_testbin.py`).
Greedy longest-match over any subset of the real vocabulary that contains every piece the
reference chose picks the same pieces, so reproducing the dump pins normalization,
pre-tokenization, WordPiece and the id runs per word against the reference's own output.
For 53 ids the dump leaves the piece string open (the split point of a word seen once);
the check runs under the canonical choice and four drawn alternates, and must hold for all.
"""
import gzip
import json
import os
import re

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TEMPLATE = os.path.join(REPO, "streaming_data_loader_amd", "assets", "bert_proxy", "tokenizer.json")


def fixture():
    with open(os.path.join(GOLDEN, "testbin_rows.json"), encoding="utf-8") as f:
        return json.load(f)


def record_runs(meta):
    """Per record: the dump's ids as `tokenizers` returns them ([CLS] ids [SEP]), a
    complete flag, and the wildcard positions (the dump holds 0 there)."""
    out, cur = [], None
    for row in meta["rows"]:
        if row[0] == 101:
            cur = []
            out.append(cur)
        cur.extend(row)
    runs = []
    for ids, rec in zip(out, meta["records"]):
        if rec["complete"]:
            ids = ids[:ids.index(102) + 1]
        runs.append((ids, rec["complete"], set(rec["wildcards"])))
    return runs


def vocab_tokens(meta, alternate=None):
    pieces = dict(meta["pieces"])
    if alternate is not None:
        pieces.update(meta["alternates"][alternate])
    inv = {int(k): v for k, v in pieces.items()}
    toks = [inv.get(i, f"[unused{i}]") for i in range(meta["vocab_size"])]
    for i, s in ((0, "[PAD]"), (100, "[UNK]"), (101, "[CLS]"), (102, "[SEP]"), (103, "[MASK]")):
        toks[i] = s
    assert len(set(toks)) == len(toks)
    return toks


def write_tokenizer(meta, outdir, alternate=None):
    """tokenizer.json (bert-base-uncased's pipeline: BertNormalizer lowercase, BertPreTokenizer,
    WordPiece ##/100, BertProcessing) + vocab.txt with the dump's pieces."""
    toks = vocab_tokens(meta, alternate)
    with open(TEMPLATE, encoding="utf-8") as f:
        tj = json.load(f)
    tj["model"]["vocab"] = {t: i for i, t in enumerate(toks)}
    os.makedirs(outdir, exist_ok=True)
    path = os.path.join(outdir, "tokenizer.json")
    with open(path, "w", encoding="utf-8") as f:
        json.dump(tj, f, ensure_ascii=False)
    with open(os.path.join(outdir, "vocab.txt"), "w", encoding="utf-8") as f:
        f.write("\n".join(toks) + "\n")
    return path


def mismatches(got, ids, complete, wild):
    """Positions where `got` (tokenizer output incl. [CLS]/[SEP]) differs from the dump."""
    if complete and len(got) != len(ids):
        return [("length", len(got), len(ids))]
    if not complete and len(got) < len(ids):
        return [("short", len(got), len(ids))]
    return [(i, got[i], ids[i]) for i in range(len(ids)) if i not in wild and got[i] != ids[i]]


ALTS = [None, 0, 1, 2, 3]


def test_fixture_shape_and_dump_texts():
    meta = fixture()
    rows = np.array(meta["rows"], np.int64)
    assert rows.shape == (8, 128)
    assert len(np.unique(rows)) == 438
    runs = record_runs(meta)
    assert [len(r[0]) for r in runs] == [339, 343, 256]
    # exactly two wildcards: position 256 of records 0 and 1 (the first slot of their third row)
    assert [sorted(r[2]) for r in runs] == [[256], [256], []]
    # the texts are the fixture's `text` fields with every JSON \uXXXX escape read as its
    # last hex digit (what the dump shows: U+2190 -> "0" = 1014, "2006 " -> 2006 ##0)
    esc = re.compile(r"\\(u[0-9a-fA-F]{4}|.)")
    texts = []
    with gzip.open(os.path.join(GOLDEN, "test.json.gz"), "rt", encoding="utf-8") as f:
        for line in f:
            obj = json.loads(esc.sub(lambda m: m.group(1)[-1] if m.group(1)[0] == "u" else m.group(0), line))
            if isinstance(obj.get("text"), str):
                texts.append(obj["text"])
    assert meta["texts"] == texts[:3]
    assert texts[0].startswith("0 August 13, 2005 August 15, 2005 2 August 14")
    assert len(meta["open_ids"]) == 53 and len(meta["alternates"]) == 4


@pytest.mark.parametrize("alt", ALTS)
def test_tokenizers_reproduces_dump(tmp_path, alt):
    tokenizers = pytest.importorskip("tokenizers")
    meta = fixture()
    tok = tokenizers.Tokenizer.from_file(write_tokenizer(meta, str(tmp_path), alt))
    for r, (ids, complete, wild) in enumerate(record_runs(meta)):
        got = tok.encode(meta["texts"][r], add_special_tokens=True).ids
        assert not mismatches(got, ids, complete, wild), (r, mismatches(got, ids, complete, wild)[:5])


@pytest.mark.parametrize("alt", ALTS)
def test_oracle_reproduces_dump(tmp_path, alt):
    import oracle_lib
    meta = fixture()
    write_tokenizer(meta, str(tmp_path), alt)
    tok = oracle_lib.Tok(vocab=os.path.join(str(tmp_path), "vocab.txt"))
    for r, (ids, complete, wild) in enumerate(record_runs(meta)):
        got = tok.encode(meta["texts"][r])
        assert not mismatches(got, ids, complete, wild), (r, mismatches(got, ids, complete, wild)[:5])


def test_oracle_batcher_reference_config(tmp_path):
    """The reference's CPU config (S=128, B=8, `masking_cases.rs:13-21`) through the oracle
    Batcher: the rows are today's framing ([CLS][CLS] ids [SEP][SEP][SEP], chunks of 128) of
    the dump's ids, so with the masks undone (labels) every dump id reappears in order."""
    import oracle_lib
    meta = fixture()
    write_tokenizer(meta, str(tmp_path))
    tok = oracle_lib.Tok(vocab=os.path.join(str(tmp_path), "vocab.txt"))
    S = 128
    planes = oracle_lib.oracle_rows(tok, meta["texts"], S, mask_length=19, seed=1234)
    check_framed_rows(meta, planes[0], planes[1], planes[3], S)


def check_framed_rows(meta, ids, am, labels, S):
    """Rows of today's Batcher over the three texts, masks undone through the labels ->
    [CLS] + ([CLS] dump ids [SEP]) + [SEP][SEP] per record, chunked at S."""
    ids, am, labels = (np.asarray(a) for a in (ids, am, labels))
    assert ((labels == -100) | (ids == 103)).all()
    orig = np.where(labels != -100, labels, ids)
    stream = []
    for g in range(ids.shape[0]):
        z = int((am[g] == 0).sum())  # the reversed-range quirk zeroes l positions of a short row
        stream += orig[g, :S if z == 0 else z].tolist()
    pos = 0
    for r, (want, complete, wild) in enumerate(record_runs(meta)):
        assert stream[pos] == 101, (r, pos)
        if complete:
            body = stream[pos + 1:pos + 1 + len(want)]
            assert stream[pos + 1 + len(want):pos + 3 + len(want)] == [102, 102]
            pos += len(want) + 3
        else:
            body = stream[pos + 1:]
        assert not mismatches(body, want, complete, wild), (r, mismatches(body, want, complete, wild)[:5])


def test_product_loader_accepts_testbin_tokenizer(tmp_path):
    """The HIP library's host-side loader (no GPU) takes the dump's vocabulary as a
    bert-base-uncased tokenizer.json: WordPiece, the special ids at their places."""
    from streaming_data_loader_amd import native
    info = native.tokenizer_info(write_tokenizer(fixture(), str(tmp_path)))
    assert (info.kind, info.vocab_size, info.unk_id) == (native.tokenizer_info(native.BERT_PROXY_TOKENIZER).kind,
                                                         30522, 100)
