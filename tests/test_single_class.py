"""Single-class task: SimpleBatcher + BertData
SingleClass (models/simple_batcher.rs:35-53, bert_data.rs:55-89) fed by
SingleClassArrowGenerator (tasks/single_class/single_arrow.rs:11-39: `text`
utf8, `label` int64 -> Label::Single(label as u32)); the batch serialises
`label` as a flat Vec<u32> with one entry per filled row (bert_data.rs:118-121).
Config: single_cases.rs (Imdb: bert-base-uncased, B=2048, S=128).

CPU tests cover the oracle (rows equal the multi-label rows of the same text:
same encode_simple framing, truncation and attention quirk), the Arrow column
reader and the frame bytes; GPU tests check the device path, the host path and
the transport frames bit-exact against the oracle."""
import pickle
import random

import numpy as np
import pytest

import oracle_lib
from streaming_data_loader_amd import arrow_io
from streaming_data_loader_amd import batcher as B


def random_items(n, seed):
    rng = random.Random(seed)
    alphabet = "abcdefghij klmnop,.;!? ÄéßİＡ中文​\t\n"
    out = []
    for _ in range(n):
        L = rng.choice([0, 1, 5, 40, 200, 700, 3000])
        out.append(("".join(rng.choice(alphabet) for _ in range(L)), rng.randrange(0, 2)))
    return out


def oracle_batches(oracle_tok, items, Bsz, S):
    ob = oracle_lib.OracleBatcherEx(oracle_lib.Encoder("bert", oracle_tok), oracle_lib.SINGLE_CLASS, Bsz, S)
    got = [r for r in (ob.push(t, [l]) for t, l in items) if r is not None]
    got.append(ob.flush())
    return got


def test_oracle_rows_match_multi_label_rows(oracle_tok):
    items = random_items(50, 1)
    sc = oracle_batches(oracle_tok, items, 8, 64)
    ml = oracle_lib.OracleBatcherEx(oracle_lib.Encoder("bert", oracle_tok), oracle_lib.MULTI_LABEL, 8, 64)
    mw = [r for r in (ml.push(t, []) for t, _ in items) if r is not None] + [ml.flush()]
    assert len(sc) == len(mw) == 7
    for a, b in zip(sc, mw):
        assert a["rows"] == b["rows"]
        for k in ("input_ids", "attention_mask", "token_type_ids"):
            np.testing.assert_array_equal(a[k], b[k])
    labels = np.concatenate([b["labels"][:b["rows"], 0] for b in sc])
    np.testing.assert_array_equal(labels, [l for _, l in items])


def test_oracle_rejects_label_count_other_than_one(oracle_tok):
    ob = oracle_lib.OracleBatcherEx(oracle_lib.Encoder("bert", oracle_tok), oracle_lib.SINGLE_CLASS, 4, 16)
    with pytest.raises(ValueError):
        ob.push("hello", [])


def test_arrow_single_class_columns():
    pa = pytest.importorskip("pyarrow")
    texts = ["a b", "", "héllo wörld", "x" * 300]
    labels = [1, 0, 7, (1 << 32) + 3]  # `as u32` wraps
    rb = pa.record_batch([pa.array(texts, pa.utf8()), pa.array(labels, pa.int64())], names=["text", "label"])
    a = arrow_io.arena_from_batch(rb, "text", "label")
    assert a.n_records == 4
    np.testing.assert_array_equal(a.labels, [1, 0, 7, 3])
    np.testing.assert_array_equal(a.label_offsets, [0, 1, 2, 3, 4])
    body = a.arena[:int(a.offsets[-1])].tobytes()
    assert body == "".join(texts).encode("utf-8")
    g = arrow_io.SingleClassArrowGenerator(rb.schema)
    t = g.get_data(rb, 2)
    assert t.data.text == "héllo wörld" and t.label.single == 7


def test_frame_label_is_flat_list():
    Bsz, S, rows = 5, 8, 3
    rng = np.random.default_rng(0)
    ids = rng.integers(0, 30000, (Bsz, S), dtype=np.int32)
    am = np.ones((Bsz, S), np.int32)
    tt = np.zeros((Bsz, S), np.int32)
    lab = np.array([[1], [0], [1], [0], [0]], np.int32)
    d = pickle.loads(oracle_lib.pickle_dataset("single-class", Bsz, S, 1, rows, ids, am, tt, lab))
    assert list(d) == ["input_ids", "attention_mask", "token_type_ids", "label"]
    assert d["label"] == [1, 0, 1] and d["input_ids"] == ids.tolist()


# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a HIP device"
    return t


@pytest.mark.gpu
@pytest.mark.parametrize("S,Bsz", [(128, 64), (100, 7)])
def test_device_path_matches_oracle(torch, native_lib, oracle_tok, S, Bsz):
    from streaming_data_loader_amd import native
    from streaming_data_loader_amd.device import DeviceBatcher, arena_from_texts
    items = random_items(500, seed=S)
    texts = [t for t, _ in items]
    arena, offs = arena_from_texts(texts)
    pad = np.zeros(arena.size + 16, np.uint8)
    pad[:arena.size] = arena
    ta = torch.from_numpy(pad).cuda()
    to = torch.from_numpy(offs.astype(np.int64)).cuda()
    tl = torch.tensor([l for _, l in items], dtype=torch.int32).cuda()
    tlo = torch.arange(len(items) + 1, dtype=torch.int64).cuda()
    db = DeviceBatcher(task=native.SDL_TASK_SINGLE_CLASS, batch_size=Bsz, sequence_length=S)
    res = db.process_labels(ta.data_ptr(), arena.size, to.data_ptr(), len(texts), tl.data_ptr(), tlo.data_ptr())
    torch.cuda.synchronize()
    assert res.rows() == len(texts) and res.label_errors() == 0
    ids, am, tt, lab = res.planes()
    want = oracle_batches(oracle_tok, items, Bsz, S)
    n = len(texts)
    np.testing.assert_array_equal(ids, np.concatenate([w["input_ids"] for w in want])[:n])
    np.testing.assert_array_equal(am, np.concatenate([w["attention_mask"] for w in want])[:n])
    np.testing.assert_array_equal(tt, np.zeros_like(tt))
    np.testing.assert_array_equal(lab[:, 0], [l for _, l in items])
    # transport frames of every batch, flushed partial included
    fr = db.pickle_frames(res, n, flush_partial=True)
    frames = fr.frames()
    assert len(frames) == len(want)
    for b, (f, w) in enumerate(zip(frames, want)):
        rows = w["rows"]
        ref = oracle_lib.pickle_dataset("single-class", Bsz, S, 1, rows, w["input_ids"], w["attention_mask"],
                                        w["token_type_ids"], w["labels"])
        assert f == ref, f"batch {b}"
        assert pickle.loads(f)["label"] == [l for _, l in items[b * Bsz:b * Bsz + rows]]
    db.close()


@pytest.mark.gpu
def test_host_path_cadence_and_arrow(torch, native_lib, oracle_tok):
    pa = pytest.importorskip("pyarrow")
    items = random_items(90, seed=5)
    sb = B.SimpleBatcher(B.ModelType.Bert, B.SingleClass(), B.BatchConfig(16, 128), B.TokenizerConfig())
    got = []
    for i, (t, l) in enumerate(items):
        ds = sb.create_sync_batch(B.SimpleTransport(B.SimpleData(t), B.Label(single=l)))
        assert (ds is not None) == ((i + 1) % 16 == 0)
        if ds is not None:
            got.append(ds)
    got.append(sb.get_working_batch())
    want = oracle_batches(oracle_tok, items, 16, 128)
    assert len(got) == len(want)
    for ds, w in zip(got, want):
        assert ds.rows == w["rows"]
        np.testing.assert_array_equal(ds.input_ids, w["input_ids"])
        np.testing.assert_array_equal(ds.attention_mask, w["attention_mask"])
        d = ds.to_dict()
        assert list(d) == ["input_ids", "attention_mask", "token_type_ids", "label"]
        np.testing.assert_array_equal(d["label"], w["labels"][:w["rows"], 0])
    # the same records as an Arrow record batch (text, label: int64)
    rb = pa.record_batch([pa.array([t for t, _ in items], pa.utf8()), pa.array([l for _, l in items], pa.int64())],
                         names=["text", "label"])
    sb2 = B.SimpleBatcher(B.ModelType.Bert, B.SingleClass(), B.BatchConfig(16, 128), B.TokenizerConfig())
    got2 = sb2.push_arrow(rb) + [sb2.get_working_batch()]
    assert len(got2) == len(want)
    for ds, w in zip(got2, want):
        np.testing.assert_array_equal(ds.input_ids, w["input_ids"])
        np.testing.assert_array_equal(ds.to_dict()["label"], w["labels"][:w["rows"], 0])
    with pytest.raises(ValueError):
        sb.create_sync_batch(B.SimpleTransport(B.SimpleData("x"), B.Label(multi=[1])))
