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
    # every shard did work, and a second push continues the global record index
    assert all(len(p) > 0 for p in per)
