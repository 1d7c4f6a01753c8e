"""GPU parity of the rand-compatible MLM mode (rng_mode 1, k_mask_rand):
device rows bit-exact against the oracle, whose StdRng / shuffle restatement
is pinned by rand's and RFC 7539's vectors (tests/test_rand_mode.py)."""
import numpy as np
import pytest

import oracle_lib
from streaming_data_loader_amd.device import DeviceBatcher
from test_gpu_parity import hard_records, run_device

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a HIP device"
    return t


@pytest.mark.parametrize("S,B,first_record,seed", [(128, 8, 0, 5), (512, 256, 1000, 1234), (1024, 16, 7, 2 ** 63 + 3),
                                                  (100, 8, 3, 11),  # (S % 8 != 0: 2-B index stores)
                                                  (2048, 4, 2, 99)])  # (RAND_MAX_S: the largest rows kernels)
def test_rand_mode_rows_match_oracle(torch, native_lib, oracle_tok, records, S, B, first_record, seed):
    rng = np.random.default_rng(S)
    texts = [records[i] for i in rng.integers(0, len(records), 300)] + hard_records(2)[:40]
    k = int(np.float32(S) * np.float32(0.15))
    db = DeviceBatcher(batch_size=B, sequence_length=S, seed=seed, rng_mode=1)
    res = run_device(torch, db, texts, first_record=first_record)
    G = res.rows()
    got = res.planes(G)
    want = oracle_lib.oracle_rows(oracle_tok, texts, S, k, 103, seed=seed, B=B, first_record=first_record,
                                  rng_mode=1)
    assert want.shape[1] == G
    for j in range(4):
        np.testing.assert_array_equal(got[j], want[j])
    # the Philox contract gives other masks on the same rows
    db0 = DeviceBatcher(batch_size=B, sequence_length=S, seed=seed, rng_mode=0)
    lab0 = run_device(torch, db0, texts, first_record=first_record).planes(G)[3]
    assert not np.array_equal(lab0, got[3])
    masked = (got[3] != -100).sum(axis=1)
    assert masked.max() <= k and masked.mean() > 0.2 * k  # pad positions (id 0) are never masked


def test_rand_mode_rejects_long_rows(native_lib):
    from streaming_data_loader_amd import native
    with pytest.raises(native.SDLError):
        DeviceBatcher(batch_size=8, sequence_length=4096, rng_mode=1)
    with pytest.raises(native.SDLError):
        DeviceBatcher(batch_size=8, sequence_length=128, rng_mode=2)


def test_rand_mode_dense_records_match_oracle(torch, native_lib, oracle_tok, records):
    """Dense records (digit and punctuation runs, ~0.5 ids per byte: many chunks per record)
    under rng_mode 1, against the oracle."""
    rng = np.random.default_rng(77)
    dense = [" ".join(str(int(x)) for x in rng.integers(0, 10, n)) + " , ." * (n // 7)
             for n in (40, 300, 700, 1500, 3000)]
    texts = [records[i] for i in rng.integers(0, len(records), 120)] + dense + [records[3]] + dense[::-1]
    S, B, seed, first = 128, 8, 99, 5
    k = int(np.float32(S) * np.float32(0.15))
    db = DeviceBatcher(batch_size=B, sequence_length=S, seed=seed, rng_mode=1)
    res = run_device(torch, db, texts, first_record=first)
    G = res.rows()
    got = res.planes(G)
    want = oracle_lib.oracle_rows(oracle_tok, texts, S, k, 103, seed=seed, B=B, first_record=first, rng_mode=1)
    assert want.shape[1] == G
    for j in range(4):
        np.testing.assert_array_equal(got[j], want[j])


@pytest.mark.parametrize("env", [{"SDL_RAND_REC0": "0"}, {"SDL_RAND_SPEC_RHO_PCT": "0"},
                                 {"SDL_RAND_SPEC_RHO_PCT": "100"}, {"SDL_RAND_SPEC_RHO_PCT": "5"}])
def test_rand_mode_mask_paths_agree(torch, native_lib, oracle_tok, records, env, monkeypatch):
    """The rows' masks come from two places (pipeline.hip rand_pre_slot): chunk 0 and guessed
    chunk-1 rows walked beside the tokenizer, the rest by k_rows' LATE pass (rand_rows16).
    Every split -- nothing beside the tokenizer, chunk 0 only, chunk 1 of every record long enough
    at 1 id per byte (every chunk-1 row there), at 0.05 ids per byte (chunk 1 guessed for few
    records) -- gives the oracle's rows."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(31)
    texts = [records[i] for i in rng.integers(0, len(records), 200)]
    texts += [" ".join(records[i] for i in rng.integers(0, len(records), 4)) for _ in range(20)]  # 3+ rows
    S, B, seed, first = 256, 16, 1234, 40
    k = int(np.float32(S) * np.float32(0.15))
    db = DeviceBatcher(batch_size=B, sequence_length=S, seed=seed, rng_mode=1)
    res = run_device(torch, db, texts, first_record=first)
    G = res.rows()
    got = res.planes(G)
    want = oracle_lib.oracle_rows(oracle_tok, texts, S, k, 103, seed=seed, B=B, first_record=first, rng_mode=1)
    assert want.shape[1] == G
    for j in range(4):
        np.testing.assert_array_equal(got[j], want[j])
