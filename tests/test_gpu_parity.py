"""GPU parity: the HIP Batcher (through the C ABI) against the CPU oracle.

Bit-exact on every id, mask and label: tokenization (WordPiece over the
BertNormalizer/BertPreTokenizer tables), framing, the <64 filter, chunking,
the attention-mask quirk and MLM masking under the RNG contract.  At the full
bench size (256 MiB arena) the checks are size-independent properties plus a
seeded sample of rows recomputed by the oracle.
"""
import os
import random

import numpy as np
import pytest

import oracle_lib
from streaming_data_loader_amd import batcher as B
from streaming_data_loader_amd import native
from streaming_data_loader_amd.device import DeviceBatcher, arena_from_texts

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a HIP device"
    return t


def to_dev(torch, texts):
    arena, offs = arena_from_texts(texts)
    pad = np.zeros(len(arena) + 16, np.uint8)
    pad[:len(arena)] = arena
    ta = torch.from_numpy(pad).cuda()[:len(arena)] if len(arena) else torch.zeros(16, dtype=torch.uint8).cuda()[:0]
    to = torch.from_numpy(offs.astype(np.int64)).cuda()
    return ta, to


def run_device(torch, db, texts, first_record=0):
    ta, to = to_dev(torch, texts)
    res = db.process(ta.data_ptr(), len(arena_from_texts(texts)[0]), to.data_ptr(), len(texts), first_record)
    torch.cuda.synchronize()
    return res


# ---------------------------------------------------------------------------
def test_stream_matches_golden_and_oracle(native_lib, records, oracle_tok):
    """Reference CPU config (BASELINE configs[0]): seq_len 128, batch 8, fixture stream."""
    g = np.load(os.path.join(GOLDEN, "mlm_s128_b8.npz"))
    gt = B.GenTokenizer(B.ModelType.Bert, B.BatchConfig(8, 128), B.Mask(19, 103), B.TokenizerConfig(), chunk=True,
                        seed=1234)
    emitted = [b for b in (gt.create_sync_batch(t) for t in records) if b is not None]
    emitted.append(gt.get_working_batch())
    assert len(emitted) == int(g["n_batches"])
    for i, ds in enumerate(emitted):
        assert ds.rows == int(g[f"b{i}_rows"])
        np.testing.assert_array_equal(ds.input_ids, g[f"b{i}_input_ids"])
        np.testing.assert_array_equal(ds.attention_mask, g[f"b{i}_attention_mask"])
        np.testing.assert_array_equal(ds.token_type_ids, g[f"b{i}_token_type_ids"])
        np.testing.assert_array_equal(ds.labels, g[f"b{i}_labels"])
        assert ds.to_dict()["labels"].shape == (ds.rows, 128)
    assert gt.get_working_batch() is None  # queue drained after the one flush


def test_push_many_matches_per_record(native_lib, records):
    cfg = (B.ModelType.Bert, B.BatchConfig(4, 128), B.Mask(19, 103), B.TokenizerConfig())
    a = B.GenTokenizer(*cfg, seed=5)
    one = [b for b in (a.create_sync_batch(t) for t in records * 2) if b is not None]
    b = B.GenTokenizer(*cfg, seed=5)
    many = b.create_sync_batches(records) + b.create_sync_batches(records)
    assert len(one) == len(many)
    for x, y in zip(one, many):
        for k in ("input_ids", "attention_mask", "token_type_ids", "labels"):
            np.testing.assert_array_equal(getattr(x, k), getattr(y, k))
    fa, fb = a.get_working_batch(), b.get_working_batch()
    assert fa.rows == fb.rows
    np.testing.assert_array_equal(fa.labels, fb.labels)


def test_batch_views_survive_block_recycling(native_lib, records):
    """DataSet arrays are zero-copy views of pinned batch blocks the handle
    recycles once a batch is released: live batches must never be reused."""
    g = B.GenTokenizer(B.ModelType.Bert, B.BatchConfig(4, 128), B.Mask(19, 103), B.TokenizerConfig(), seed=9)
    first = g.create_sync_batches(records)
    assert len(first) > 4
    ptrs = {ds.input_ids.ctypes.data for ds in first}
    assert len(ptrs) == len(first)  # one block per live batch
    keep = first[::2]
    snap = [(ds.input_ids.copy(), ds.attention_mask.copy(), ds.token_type_ids.copy(), ds.labels.copy()) for ds in keep]
    del first
    for _ in range(3):  # released blocks get reused by these calls
        more = g.create_sync_batches(records)
        del more
    for ds, (i, a, t, l) in zip(keep, snap):
        np.testing.assert_array_equal(ds.input_ids, i)
        np.testing.assert_array_equal(ds.attention_mask, a)
        np.testing.assert_array_equal(ds.token_type_ids, t)
        np.testing.assert_array_equal(ds.labels, l)


def test_b1_cadence_drops_like_reference(native_lib, records, oracle_tok):
    """B=1 (the reference's test config): a record yielding k rows queues k
    batches, only one is emitted per call and one on flush (gen_batcher.rs:86-91)."""
    gt = B.GenTokenizer(B.ModelType.Bert, B.BatchConfig(1, 128), B.Mask(19, 103), B.TokenizerConfig(), seed=3)
    ob = oracle_lib.OracleBatcher(oracle_tok, 1, 128, 19, 103, seed=3)
    for t in records[:10]:
        x, y = gt.create_sync_batch(t), ob.push(t)
        assert (x is None) == (y is None)
        if x is not None:
            np.testing.assert_array_equal(x.input_ids, y[0][0])
            np.testing.assert_array_equal(x.labels, y[0][3])
    x, y = gt.get_working_batch(), ob.flush()
    np.testing.assert_array_equal(x.input_ids, y[0][0])


# ---------------------------------------------------------------------------
def hard_records(seed=0):
    """Records that stress the tokenizer: every golden edge case, plus long
    and pathological words, DEL runs, specials and multi-byte runs."""
    import json
    cases = [c["text"] for c in json.load(open(os.path.join(GOLDEN, "bert_ids.json"), encoding="utf-8"))["cases"]]
    rng = random.Random(seed)
    extra = ["a" * 5000, "é" * 3000, "x\x00" * 3000, "[SEP]" * 900, "中" * 2000, "word " * 2000,
             "tokenization" * 30, ("ab​" * 40) + " tail", "!" * 5000, "\U0001f600" * 1500,
             " ".join("supercalifragilistic" for _ in range(300)), "\t\n " * 100 + "end"]
    out = cases + extra
    rng.shuffle(out)
    return out


def framed_rows(oracle_tok, texts, S):
    """Expected input_ids rows with no masking and no length filter."""
    rows = []
    for t in texts:
        ids = [101] + oracle_tok.encode(t) + [102, 102]
        for o in range(0, len(ids), S):
            r = np.zeros(S, np.int32)
            c = ids[o:o + S]
            r[:len(c)] = c
            rows.append(r)
    return np.array(rows, np.int32).reshape(-1, S)


def test_tokenizer_on_hard_records(torch, native_lib, oracle_tok):
    texts = hard_records()
    db = DeviceBatcher(batch_size=16, sequence_length=128, mask_length=0, min_ids=0)
    res = run_device(torch, db, texts)
    ids, am, tt, lab = res.planes()
    want = framed_rows(oracle_tok, texts, 128)
    assert ids.shape == want.shape
    bad = np.nonzero((ids != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} rows differ, first {bad[:5]}"
    assert (lab == -100).all()


def test_canonical_ordering_on_device(torch, native_lib):
    """NFD canonical ordering of kept combining marks (tests/golden/
    bert_marks_ids.json, widened vocab): every golden case as its own record,
    then the cases joined into long records so mark runs straddle chunk seams
    (checked against the oracle, pinned by the same goldens)."""
    import json
    g = json.load(open(os.path.join(GOLDEN, "bert_marks_ids.json"), encoding="utf-8"))
    tj = os.path.join(GOLDEN, "bert_marks", "tokenizer.json")
    tok = oracle_lib.Tok(vocab=os.path.join(GOLDEN, "bert_marks", "vocab.txt"))
    texts = [c["text"] for c in g["cases"]]

    class Golden:
        ids = {c["text"]: c["ids"] for c in g["cases"]}

        def encode(self, t):
            return self.ids[t]

    rng = random.Random(7)
    long_texts = []
    for _ in range(24):
        sel = rng.sample(texts, 120)
        long_texts.append(rng.choice(["", " ", "x"]).join(sel))
    for batch, want_tok in ((texts, Golden()), (long_texts, tok)):
        db = DeviceBatcher(batch_size=16, sequence_length=128, mask_length=0, min_ids=0, tokenizer=tj)
        ids = run_device(torch, db, batch).planes()[0]
        want = framed_rows(want_tok, batch, 128)
        assert ids.shape == want.shape
        bad = np.nonzero((ids != want).any(axis=1))[0]
        assert bad.size == 0, f"{bad.size} rows differ, first {bad[:5]}"
        db.close()


@pytest.mark.parametrize("feature", ["[SEP]", "é", "中", "\U0001f600", "\x00", "​", " ", "!", "supercalifragilisticexpialidocious"])
def test_chunk_boundary_straddle(torch, native_lib, oracle_tok, feature):
    """Put `feature` across every position near the 4096-byte chunk seams,
    and record boundaries on the seams themselves."""
    texts = []
    for shift in range(-8, 9):
        left = "ab " * ((4096 + shift) // 3) + "c" * ((4096 + shift) % 3)
        texts.append(left + feature + " zz" + feature + "q")
    # a record boundary exactly on a chunk boundary, and empty records there
    texts += ["x" * 4096, "", "", "y" * 4095, "z" * 4097, ""]
    db = DeviceBatcher(batch_size=8, sequence_length=256, mask_length=0, min_ids=0)
    res = run_device(torch, db, texts)
    ids = res.planes()[0]
    want = framed_rows(oracle_tok, texts, 256)
    np.testing.assert_array_equal(ids, want)


def test_mlm_rows_match_oracle_s512(torch, native_lib, oracle_tok, records):
    """BASELINE configs[1] shape: mlm S=512 B=256, bit-exact vs the oracle."""
    rng = np.random.default_rng(0x5D1B)
    texts = [records[i] for i in rng.integers(0, len(records), 600)] + hard_records(1)
    db = DeviceBatcher(batch_size=256, sequence_length=512, seed=1234)
    res = run_device(torch, db, texts, first_record=1000)
    G = res.rows()
    ids, am, tt, lab = res.planes(G)
    want = oracle_lib.oracle_rows(oracle_tok, texts, 512, 76, 103, seed=1234, B=256, first_record=1000)
    assert want.shape[1] == G
    for j, got in enumerate((ids, am, tt, lab)):
        np.testing.assert_array_equal(got, want[j])
    # pad rows of the last batch hold the initial values
    Gp = -(-G // 256) * 256
    ids2, am2, tt2, lab2 = res.planes(Gp)
    assert (ids2[G:] == 0).all() and (am2[G:] == 1).all() and (lab2[G:] == -100).all()


def test_clm_rows(torch, native_lib, oracle_tok, records):
    """GptData::put_data semantics (labels = ids, quirk range -100/0) over the
    WordPiece path (byte-BPE tokenization is a later row)."""
    db = DeviceBatcher(task=native.SDL_TASK_CLM, batch_size=8, sequence_length=128)
    res = run_device(torch, db, records)
    ids, am, tt, lab = res.planes()
    assert tt is None
    want = framed_rows(oracle_tok, [t for t in records if len(oracle_tok.encode(t)) + 3 >= 64], 128)
    np.testing.assert_array_equal(ids, want)
    for i in range(ids.shape[0]):
        l = 128 - int((am[i] == 0).sum()) if (am[i] == 0).any() else 128
        # quirk: positions S-l..S-1 of a short row get attention 0 / label -100
        nz = int((want[i] != 0).sum())
        if nz < 128:
            assert (am[i][128 - nz:] == 0).all() and (am[i][:128 - nz] == 1).all()
        assert ((lab[i] == -100) == (am[i] == 0)).all()
        assert (lab[i][am[i] == 1] == ids[i][am[i] == 1]).all()


# ---------------------------------------------------------------------------
def bench_arena(records, nbytes, seed=0x5D1B):
    """The bench workload: fixture records tiled in seeded permutations."""
    blobs = [r.encode("utf-8") for r in records]
    rng = np.random.default_rng(seed)
    order, total = [], 0
    while total < nbytes:
        for i in rng.permutation(len(blobs)):
            order.append(int(i))
            total += len(blobs[i])
            if total >= nbytes:
                break
    lens = np.array([len(blobs[i]) for i in order], np.uint64)
    offs = np.zeros(len(order) + 1, np.uint64)
    np.cumsum(lens, out=offs[1:])
    arena = np.concatenate([np.frombuffer(blobs[i], np.uint8) for i in order])
    return arena, offs, order


def test_full_size_properties(torch, native_lib, oracle_tok, records):
    arena, offs, order = bench_arena(records, 256 << 20)
    ta = torch.from_numpy(np.concatenate([arena, np.zeros(16, np.uint8)])).cuda()
    to = torch.from_numpy(offs.astype(np.int64)).cuda()
    db = DeviceBatcher(batch_size=256, sequence_length=512, seed=1234)
    res = db.process(ta.data_ptr(), len(arena), to.data_ptr(), len(order))
    torch.cuda.synchronize()
    # per record: ids and rows are fixed by the record's text
    n_ids = np.array([len(oracle_tok.encode(r)) - 2 for r in records], np.int64)
    framed = n_ids + 5
    rows_of = np.where(framed >= 64, -(-framed // 512), 0)
    want_rows = rows_of[order]
    got_rows = res.record_rows()
    np.testing.assert_array_equal(got_rows, want_rows)
    assert res.tokens() == int(n_ids[order].sum())
    G = res.rows()
    assert G == int(want_rows.sum())
    ids, am, tt, lab = res.planes(G)
    masked = lab != -100
    assert (ids[masked] == 103).all() and (tt == 0).all()
    full = am.all(axis=1)
    assert (masked[full].sum(axis=1) == 76).all()
    assert (masked.sum(axis=1) <= 76).all()
    # seeded sample of records recomputed by the oracle, global record index kept
    row_off = np.concatenate([[0], np.cumsum(got_rows)])
    for r in np.random.default_rng(7).choice(len(order), 24, replace=False):
        r = int(r)
        if got_rows[r] == 0:
            continue
        want = oracle_lib.oracle_rows(oracle_tok, [records[order[r]]], 512, 76, 103, seed=1234, B=256, first_record=r)
        sl = slice(int(row_off[r]), int(row_off[r + 1]))
        for j, got in enumerate((ids, am, tt, lab)):
            np.testing.assert_array_equal(got[sl], want[j])


@pytest.mark.parametrize("segments", [2, 3, 7])
def test_pipelined_segments_match_oracle(torch, native_lib, oracle_tok, records, segments, monkeypatch):
    """The WordPiece path cut into pipelined segments (tokenize on the caller's
    stream, scans/compaction/records/rows of finished segments on a second
    stream): same rows as the oracle, pad rows included, for segment counts
    whose cuts fall inside records; mlm and multi-label."""
    monkeypatch.setenv("SDL_SEGMENTS", str(segments))
    monkeypatch.setenv("SDL_SEG_MIN_CHUNKS", "16")
    rng = np.random.default_rng(segments)
    texts = [records[i] for i in rng.integers(0, len(records), 400)] + hard_records(segments)
    db = DeviceBatcher(batch_size=32, sequence_length=512, seed=99)
    res = run_device(torch, db, texts, first_record=17)
    G = res.rows()
    Gp = -(-G // 32) * 32
    ids, am, tt, lab = res.planes(Gp)
    want = oracle_lib.oracle_rows(oracle_tok, texts, 512, 76, 103, seed=99, B=32, first_record=17)
    assert want.shape[1] == G
    for j, got in enumerate((ids, am, tt, lab)):
        np.testing.assert_array_equal(got[:G], want[j])
    assert (ids[G:] == 0).all() and (am[G:] == 1).all() and (lab[G:] == -100).all()
    assert int(res.record_rows().sum()) == G
    # the same arena twice through one handle: buffers reused across calls
    res2 = run_device(torch, db, texts, first_record=17)
    assert res2.rows() == G
    np.testing.assert_array_equal(res2.planes(G)[0], want[0])


def test_zero_copy_tensors_and_batches(torch, native_lib, oracle_tok, records):
    """DeviceResult.tensors() / batches(): zero-copy device views of the planes
    (the consumer without serde_pickle) equal the copied planes and the oracle's
    batches, the last one padded with initial values; multi-label's float32 labels."""
    texts = records[:300]
    db = DeviceBatcher(batch_size=32, sequence_length=128, seed=11)
    res = run_device(torch, db, texts, first_record=5)
    G = res.rows()
    want = oracle_lib.oracle_rows(oracle_tok, texts, 128, 19, 103, seed=11, B=32, first_record=5)
    t = res.tensors()
    assert set(t) == {"input_ids", "attention_mask", "token_type_ids", "labels"}
    for j, k in enumerate(("input_ids", "attention_mask", "token_type_ids", "labels")):
        assert t[k].is_cuda and t[k].dtype == torch.int32 and tuple(t[k].shape) == (G, 128)
        np.testing.assert_array_equal(t[k].cpu().numpy(), want[j])
    bs = res.batches()
    assert len(bs) == -(-G // 32) and sum(b["rows"] for b in bs) == G
    for b_i, b in enumerate(bs):
        assert tuple(b["input_ids"].shape) == (32, 128)
        r = b["rows"]
        np.testing.assert_array_equal(b["input_ids"][:r].cpu().numpy(), want[0][b_i * 32:b_i * 32 + r])
    last = bs[-1]
    if last["rows"] < 32:
        assert (last["input_ids"][last["rows"]:] == 0).all() and (last["labels"][last["rows"]:] == -100).all()
    db.close()
    ml = DeviceBatcher(task=native.SDL_TASK_MULTI_LABEL, batch_size=16, sequence_length=128, number_labels=9)
    arena, offs = arena_from_texts(texts[:40])
    labels = np.array([i % 9 for i in range(40)], np.uint32)
    loff = np.arange(41, dtype=np.uint64)
    ta = torch.from_numpy(np.concatenate([arena, np.zeros(16, np.uint8)])).cuda()
    to = torch.from_numpy(offs.astype(np.int64)).cuda()
    tl = torch.from_numpy(labels.astype(np.int32)).cuda()
    tlo = torch.from_numpy(loff.astype(np.int64)).cuda()
    r2 = ml.process_labels(ta.data_ptr(), len(arena), to.data_ptr(), 40, tl.data_ptr(), tlo.data_ptr())
    torch.cuda.synchronize()
    t2 = r2.tensors()
    assert t2["labels"].dtype == torch.float32 and tuple(t2["labels"].shape) == (r2.rows(), 9)
    np.testing.assert_array_equal(t2["labels"].cpu().numpy(), r2.planes()[3])
    ml.close()
