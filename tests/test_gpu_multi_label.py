"""GPU parity for the multi-label task (SimpleBatcher + BertData MultiLabel,
simple_batcher.rs:35-53, bert_data.rs:55-89) fed from Arrow records
(MultiArrowGenerator, multi_arrow.rs:11-41): ids, attention quirk and the
f32 multi-hot labels bit-exact against the golden npz and the CPU oracle."""
import os
import random

import numpy as np
import pytest

import oracle_lib
from streaming_data_loader_amd import arrow_io
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


def fixture_items():
    items, batches = [], list(arrow_io.read_stream(os.path.join(GOLDEN, "multi_label.arrow")))
    for b in batches:
        gen = arrow_io.MultiArrowGenerator(b.schema)
        items += [gen.get_data(b, i) for i in range(b.num_rows)]
    return items, batches


def golden_batches():
    g = np.load(os.path.join(GOLDEN, "multi_label_s128_b8.npz"))
    return [{k: g[f"b{i}_{k}"] for k in ("input_ids", "attention_mask", "token_type_ids", "labels", "rows")}
            for i in range(int(g["n_batches"]))]


def assert_ds(ds, want, msg=""):
    assert ds.rows == int(want["rows"]), msg
    np.testing.assert_array_equal(ds.input_ids, want["input_ids"], err_msg=msg)
    np.testing.assert_array_equal(ds.attention_mask, want["attention_mask"], err_msg=msg)
    np.testing.assert_array_equal(ds.token_type_ids, want["token_type_ids"], err_msg=msg)
    assert ds.labels.dtype == np.float32
    np.testing.assert_array_equal(ds.labels, want["labels"], err_msg=msg)


def make_simple(B_=8, S=128):
    return B.SimpleBatcher(B.ModelType.Bert, B.MultiLabel(9), B.BatchConfig(B_, S), B.TokenizerConfig())


def test_per_record_cadence_matches_golden(native_lib):
    items, _ = fixture_items()
    sb = make_simple()
    got = []
    for i, t in enumerate(items):
        ds = sb.create_sync_batch(t)
        assert (ds is not None) == ((i + 1) % 8 == 0)  # the filling call returns the batch
        if ds is not None:
            got.append(ds)
    got.append(sb.get_working_batch())
    want = golden_batches()
    assert len(got) == len(want)
    for i, (ds, w) in enumerate(zip(got, want)):
        assert_ds(ds, w, f"batch {i}")
    d = got[0].to_dict()
    assert d["labels"].shape == (8, 9) and set(d) == {"input_ids", "attention_mask", "token_type_ids", "labels"}
    e = sb.get_working_batch()  # SimpleBatcher always has a working batch
    assert e is not None and e.rows == 0


def test_arrow_batches_match_golden(native_lib):
    _, batches = fixture_items()
    sb = make_simple()
    got = []
    for b in batches:
        got += sb.push_arrow(b)
    got.append(sb.get_working_batch())
    want = golden_batches()
    assert len(got) == len(want)
    for i, (ds, w) in enumerate(zip(got, want)):
        assert_ds(ds, w, f"batch {i}")


def test_bad_label_index_is_an_error(native_lib):
    sb = make_simple()
    with pytest.raises(native.SDLError):
        sb.create_sync_batch(B.SimpleTransport(B.SimpleData("hello"), B.Label(multi=[9])))
    with pytest.raises(ValueError):
        sb.create_sync_batch(B.SimpleTransport(B.SimpleData("hello"), None))


def random_items(n, seed):
    rng = random.Random(seed)
    alphabet = "abcdefghij klmnop,.;!? ÄéßİＡ中文​\t\n"
    items = []
    for _ in range(n):
        L = rng.choice([0, 1, 5, 40, 200, 700, 3000])
        text = "".join(rng.choice(alphabet) for _ in range(L))
        labels = sorted(rng.sample(range(9), rng.randint(0, 4)))
        items.append((text, labels))
    return items


@pytest.mark.parametrize("S,Bsz,segments", [(128, 64, 1), (512, 16, 1), (100, 7, 1), (128, 64, 5), (100, 7, 3)])
def test_device_path_matches_oracle(torch, native_lib, oracle_tok, S, Bsz, segments, monkeypatch):
    """sdl_process_device_labels on ragged random records vs the oracle
    (segments > 1: the pipelined two-stream path)."""
    monkeypatch.setenv("SDL_SEGMENTS", str(segments))
    monkeypatch.setenv("SDL_SEG_MIN_CHUNKS", "16")
    items = random_items(600, seed=S)
    texts = [t for t, _ in items]
    arena, offs = arena_from_texts(texts)
    pad = np.zeros(arena.size + 16, np.uint8)
    pad[:arena.size] = arena
    vals, loffs = B._pack_labels([l for _, l in items])
    ta = torch.from_numpy(pad).cuda()
    to = torch.from_numpy(offs.astype(np.int64)).cuda()
    tl = torch.from_numpy(vals.astype(np.int32)).cuda()
    tlo = torch.from_numpy(loffs.astype(np.int64)).cuda()
    db = DeviceBatcher(task=native.SDL_TASK_MULTI_LABEL, batch_size=Bsz, sequence_length=S)
    res = db.process_labels(ta.data_ptr(), arena.size, to.data_ptr(), len(texts), tl.data_ptr(), tlo.data_ptr())
    torch.cuda.synchronize()
    assert res.rows() == len(texts) and res.label_errors() == 0
    ids, am, tt, lab = res.planes()
    ob = oracle_lib.OracleBatcherEx(oracle_lib.Encoder("bert", oracle_tok), oracle_lib.MULTI_LABEL, Bsz, S)
    want = [r for r in (ob.push(t, l) for t, l in items) if r is not None]
    last = ob.flush()
    want.append(last)
    wi = np.concatenate([w["input_ids"] for w in want])[:len(texts)]
    wa = np.concatenate([w["attention_mask"] for w in want])[:len(texts)]
    wl = np.concatenate([w["labels_f32"] for w in want])[:len(texts)]
    np.testing.assert_array_equal(ids, wi)
    np.testing.assert_array_equal(am, wa)
    np.testing.assert_array_equal(tt, np.zeros_like(tt))
    np.testing.assert_array_equal(lab, wl)
    # padding rows of the last batch hold the initial values
    Gpad = -(-len(texts) // Bsz) * Bsz
    if Gpad > len(texts):
        ids2, am2, _, lab2 = res.planes(Gpad)
        assert (ids2[len(texts):] == 0).all() and (am2[len(texts):] == 1).all() and (lab2[len(texts):] == 0).all()


def test_device_path_counts_bad_labels(torch, native_lib):
    texts = ["one", "two", "three"]
    arena, offs = arena_from_texts(texts)
    pad = np.zeros(arena.size + 16, np.uint8)
    pad[:arena.size] = arena
    ta = torch.from_numpy(pad).cuda()
    to = torch.from_numpy(offs.astype(np.int64)).cuda()
    tl = torch.tensor([1, 9, 2, 100, 3], dtype=torch.int32).cuda()
    tlo = torch.tensor([0, 2, 4, 5], dtype=torch.int64).cuda()
    db = DeviceBatcher(task=native.SDL_TASK_MULTI_LABEL, batch_size=4, sequence_length=16)
    res = db.process_labels(ta.data_ptr(), arena.size, to.data_ptr(), 3, tl.data_ptr(), tlo.data_ptr())
    torch.cuda.synchronize()
    assert res.label_errors() == 2
    lab = res.planes()[3]
    assert lab[0].tolist() == [0, 1, 0, 0, 0, 0, 0, 0, 0]
    assert lab[1].tolist() == [0, 0, 1, 0, 0, 0, 0, 0, 0]
    assert lab[2].tolist() == [0, 0, 0, 1, 0, 0, 0, 0, 0]
