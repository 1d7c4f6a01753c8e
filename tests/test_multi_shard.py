"""Several GPUs over one record stream (sdl_shard_records + sdl_multi_*).

CPU: the shard plan (host only) cuts the stream into contiguous byte-balanced record
ranges, and -- because masks depend only on (seed, global record index, chunk) -- the rows
of N shards, each a Batcher of its own, concatenate to the rows of one Batcher over the
whole stream (checked on the C oracle, which the HIP path is bit-exact to).
GPU: ShardedGenTokenizer drives three handles (on one device here) from one push and gives
the same rows as one GenTokenizer over the stream, per shard in record order."""
import os

import numpy as np
import pytest

import oracle_lib
from streaming_data_loader_amd import native

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def stream(records, nbytes, seed=0x5D1B):
    import sys
    sys.path.insert(0, REPO)
    import bench
    order = bench.build_order(records, nbytes, seed)
    texts = [records[i] for i in order]
    offs = np.zeros(len(texts) + 1, np.uint64)
    np.cumsum([len(t.encode()) for t in texts], out=offs[1:])
    return texts, offs


@pytest.mark.parametrize("n", [1, 2, 3, 7])
def test_shard_plan_is_contiguous_and_byte_balanced(native_lib, records, n):
    texts, offs = stream(records, 200_000)
    b = native.shard_records(offs, n)
    assert b[0] == 0 and b[-1] == len(texts) and (np.diff(b.astype(np.int64)) >= 0).all()
    total = int(offs[-1])
    biggest = max(len(t.encode()) for t in texts)
    for k in range(n):
        # bound k is the first record starting at or past k * total / n
        assert int(offs[b[k]]) >= k * total // n
        assert b[k] == 0 or int(offs[b[k] - 1]) < k * total // n
        got = int(offs[b[k + 1]] - offs[b[k]])
        assert abs(got - total / n) <= biggest


def test_shard_plan_edge_cases(native_lib):
    offs = np.array([0, 10, 10, 10, 40], np.uint64)
    assert native.shard_records(offs, 1).tolist() == [0, 4]
    assert native.shard_records(offs, 2).tolist() == [0, 4, 4]  # no record starts at or past 20
    assert native.shard_records(offs, 4).tolist() == [0, 1, 4, 4, 4]
    assert native.shard_records(offs, 8).tolist()[-1] == 4
    assert native.shard_records(np.zeros(1, np.uint64), 3).tolist() == [0, 0, 0, 0]
    with pytest.raises(native.SDLError):
        native.shard_records(np.array([0, 5, 3], np.uint64), 2)


@pytest.mark.parametrize("n", [2, 3])
def test_shards_rows_equal_whole_stream_rows(native_lib, records, n):
    texts, offs = stream(records, 120_000)
    S, B, k = 128, 8, 19
    tok = oracle_lib.Tok()
    whole = oracle_lib.oracle_rows(tok, texts, S, k, seed=1234, B=B)
    b = native.shard_records(offs, n)
    parts = [oracle_lib.oracle_rows(tok, texts[int(b[i]):int(b[i + 1])], S, k, seed=1234, B=B,
                                    first_record=int(b[i])) for i in range(n)]
    np.testing.assert_array_equal(np.concatenate(parts, axis=1), whole)


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a HIP device"
    return t


def _rows(batches):
    """The filled rows of a batch sequence, per plane."""
    keys = ("input_ids", "attention_mask", "token_type_ids", "labels")
    return [np.concatenate([np.asarray(getattr(d, k))[:d.rows] if k != "labels" else np.asarray(d.labels)[:d.rows]
                            for d in batches]) for k in keys]


@pytest.mark.gpu
@pytest.mark.parametrize("rng_mode", [0, 1])
def test_sharded_gen_tokenizer_matches_one_handle(torch, native_lib, records, rng_mode):
    from streaming_data_loader_amd import BatchConfig, GenTokenizer, Mask, ModelType, ShardedGenTokenizer, \
        TokenizerConfig
    texts, offs = stream(records, 400_000)
    cfg = (ModelType.Bert, BatchConfig(8, 128), Mask(19, 103), TokenizerConfig())
    one = GenTokenizer(*cfg, chunk=True, seed=1234, rng_mode=rng_mode)
    ref = one.create_sync_batches(texts)
    last = one.get_working_batch()
    while last is not None and last.rows:
        ref.append(last)
        last = one.get_working_batch()
    sh = ShardedGenTokenizer(*cfg, devices=[0, 0, 0], seed=1234, rng_mode=rng_mode)
    per = sh.create_sync_batches(texts)
    got = []
    for k in range(3):
        got += per[k]
        last = sh.get_working_batch(k)
        while last is not None and last.rows:
            got.append(last)
            last = sh.get_working_batch(k)
    want_rows, got_rows = _rows(ref), _rows(got)
    for w, g in zip(want_rows, got_rows):
        np.testing.assert_array_equal(g, w)
    # every shard did work (a second push: test_two_pushes_continue_the_global_record_index)
    assert all(len(p) > 0 for p in per)


def _drain_shard(sh, per, k):
    got = list(per[k])
    last = sh.get_working_batch(k)
    while last is not None and last.rows:
        got.append(last)
        last = sh.get_working_batch(k)
    return got


@pytest.mark.gpu
def test_two_pushes_continue_the_global_record_index(torch, native_lib, records):
    """Two sdl_multi_push_many calls: shard k holds push 1's range k then push 2's range k,
    each record keyed by its global index (push 2's records from n1 on).  Every shard's rows
    equal an oracle Batcher fed the same records with the same global indices."""
    from streaming_data_loader_amd import BatchConfig, Mask, ModelType, ShardedGenTokenizer, TokenizerConfig
    texts, _ = stream(records, 300_000)
    n1 = len(texts) // 3
    p1, p2 = texts[:n1], texts[n1:]
    S, B, k_mask, seed = 128, 8, 19, 1234
    sh = ShardedGenTokenizer(ModelType.Bert, BatchConfig(B, S), Mask(k_mask, 103), TokenizerConfig(),
                             devices=[0, 0, 0], seed=seed)
    per1 = sh.create_sync_batches(p1)
    per2 = sh.create_sync_batches(p2)
    tok = oracle_lib.Tok()
    b1 = native.shard_records(np.cumsum([0] + [len(t.encode()) for t in p1]).astype(np.uint64), 3)
    b2 = native.shard_records(np.cumsum([0] + [len(t.encode()) for t in p2]).astype(np.uint64), 3)
    for k in range(3):
        got = _drain_shard(sh, [a + b for a, b in zip(per1, per2)], k)
        ob = oracle_lib.OracleBatcher(tok, B, S, k_mask, 103, seed)
        planes = []
        for base, part, b in ((0, p1, b1), (n1, p2, b2)):
            ob.set_next_record(base + int(b[k]))
            for t in part[int(b[k]):int(b[k + 1])]:
                r = ob.push(t)
                if r is not None:
                    planes.append(r[0][:, :r[1]])
        while True:
            r = ob.flush()
            if r is None:
                break
            planes.append(r[0][:, :r[1]])
        want = np.concatenate(planes, axis=1)
        for w, g in zip(want, _rows(got)):
            np.testing.assert_array_equal(g, w)


@pytest.mark.gpu
def test_sharded_multi_label_matches_one_simple_batcher(torch, native_lib, records):
    """sdl_multi over the multi-label task (SimpleBatcher, Label::Multi): the label values
    are passed whole and each shard reads its records' slice through label_offsets; the
    shards' rows (full batches + the flushed partial) concatenate to one SimpleBatcher's."""
    import random
    from streaming_data_loader_amd import BatchConfig, ModelType, ShardedGenTokenizer, TokenizerConfig
    from streaming_data_loader_amd import batcher as Bt
    rng = random.Random(9)
    texts = [records[rng.randrange(len(records))][:rng.choice([5, 80, 400, 3000])] for _ in range(300)]
    labs = [sorted(rng.sample(range(9), rng.randint(0, 4))) for _ in texts]
    blobs = [t.encode() for t in texts]
    offs = np.zeros(len(blobs) + 1, np.uint64)
    np.cumsum([len(b) for b in blobs], out=offs[1:])
    arena = np.frombuffer(b"".join(blobs) + b"\0" * 16, np.uint8)
    vals = np.array([x for l in labs for x in l], np.uint32)
    loffs = np.zeros(len(labs) + 1, np.uint64)
    np.cumsum([len(l) for l in labs], out=loffs[1:])
    one = Bt.SimpleBatcher(ModelType.Bert, Bt.MultiLabel(9), BatchConfig(16, 128), TokenizerConfig())
    ref = one.push_arena(arena, offs, vals, loffs)
    last = one.get_working_batch()
    if last is not None and last.rows:
        ref.append(last)
    sh = ShardedGenTokenizer(ModelType.Bert, BatchConfig(16, 128), Bt.MultiLabel(9), TokenizerConfig(),
                             devices=[0, 0, 0], chunk=False)
    per = sh.push_arena(arena, offs, vals, loffs)
    got = []
    for k in range(3):
        got += per[k]
        last = sh.get_working_batch(k)
        if last is not None and last.rows:
            got.append(last)
    keys = ("input_ids", "attention_mask", "token_type_ids", "labels")
    for key in keys:
        w = np.concatenate([np.asarray(getattr(d, key))[:d.rows] for d in ref])
        g = np.concatenate([np.asarray(getattr(d, key))[:d.rows] for d in got])
        np.testing.assert_array_equal(g, w)
    assert all(len(p) > 0 for p in per)


@pytest.mark.gpu
def test_a_failed_shard_poisons_the_multi_handle(torch, native_lib, records):
    """A label index >= number_labels fails its shard: the call fails, and later pushes are
    refused (SDL_ERR_STATE) since the other shards already committed their batches."""
    from streaming_data_loader_amd import BatchConfig, ModelType, ShardedGenTokenizer, TokenizerConfig
    from streaming_data_loader_amd import batcher as Bt
    blobs = [r.encode() for r in records[:12]]
    offs = np.zeros(len(blobs) + 1, np.uint64)
    np.cumsum([len(b) for b in blobs], out=offs[1:])
    arena = np.frombuffer(b"".join(blobs) + b"\0" * 16, np.uint8)
    vals = np.array([1] * 11 + [9], np.uint32)  # the last record (shard 1) carries a bad label
    loffs = np.arange(13, dtype=np.uint64)
    sh = ShardedGenTokenizer(ModelType.Bert, BatchConfig(2, 128), Bt.MultiLabel(9), TokenizerConfig(),
                             devices=[0, 0], chunk=False)
    with pytest.raises(native.SDLError):
        sh.push_arena(arena, offs, vals, loffs)
    with pytest.raises(native.SDLError, match="earlier push failed"):
        sh.push_arena(arena, offs, np.ones(12, np.uint32), loffs)
