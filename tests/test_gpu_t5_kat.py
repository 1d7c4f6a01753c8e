"""The HIP path against the reference's t5 known-answer vector (see tests/test_t5_kat.py):
`/root/reference/python/test_t5.py:3-7`, t5-small ids of "I am here to save the day. The
dog is done with the food.", through the t5 proxy tokenizer with the KAT's pieces at their
t5-small ids (tests/golden/make_t5_kat_vocab.py).

  * tokenizer ids per record (clm rows over the t5 tokenizer, no length filter): the KAT
    text alone, and embedded at every offset around a 1 KiB chunk seam, each record
    giving encode_mask's [</s>] + KAT + [</s>] (tokenizer_wrapper.rs:125-130);
  * span rows (T5Data::put_data, configs[2]'s task) over records built from the sentence,
    in both RNG modes, equal to the oracle's rows under the same tokenizer -- whose ids the
    CPU test pins to the KAT."""
import os
import sys

import numpy as np
import pytest

import oracle_lib
from streaming_data_loader_amd import native
from streaming_data_loader_amd.device import DeviceBatcher

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_t5_kat_vocab as kat  # noqa: E402


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a HIP device"
    return t


@pytest.fixture(scope="module")
def kat_tokenizer(tmp_path_factory):
    import json
    path = os.path.join(str(tmp_path_factory.mktemp("t5_kat")), "tokenizer.json")
    with open(path, "w", encoding="utf-8") as f:
        json.dump(kat.build(), f, ensure_ascii=False)
    return path


def _arena(torch, texts):
    blobs = [t.encode("utf-8") for t in texts]
    offs = np.zeros(len(blobs) + 1, np.uint64)
    np.cumsum([len(b) for b in blobs], out=offs[1:])
    arena = np.zeros(int(offs[-1]) + 16, np.uint8)
    arena[:int(offs[-1])] = np.frombuffer(b"".join(blobs), np.uint8)
    return torch.from_numpy(arena).cuda(), torch.from_numpy(offs.astype(np.int64)).cuda(), int(offs[-1])


def _record_ids(res, S, n_records):
    ids, am, _, _ = res.planes()
    per = res.record_rows()
    out, g = [], 0
    for r in range(n_records):
        seq = []
        for _ in range(int(per[r])):
            z = int((am[g] == 0).sum())
            seq += ids[g, :S if z == 0 else z].tolist()
            g += 1
        out.append(seq)
    return out


def test_device_ids_reproduce_the_kat(torch, native_lib, kat_tokenizer):
    S = 128
    # the sentence alone, then behind fillers that put it across the first 1 KiB chunk seam
    texts = [kat.KAT_TEXT]
    for k in range(0, 64, 3):
        cur = sum(len(t.encode()) for t in texts)
        texts += ["x" * (((1024 - 40 + k - 1 - cur % 1024 + 1024) % 1024) or 1), kat.KAT_TEXT]
    db = DeviceBatcher(task=native.SDL_TASK_CLM, batch_size=8, sequence_length=S, min_ids=0,
                       tokenizer=kat_tokenizer)
    ta, to, n = _arena(torch, texts)
    res = db.process(ta.data_ptr(), n, to.data_ptr(), len(texts))
    torch.cuda.synchronize()
    assert res.tokenize_errors() == 0
    got = _record_ids(res, S, len(texts))
    want = [1] + kat.KAT_IDS + [1]
    kat_records = [r for r, t in enumerate(texts) if t == kat.KAT_TEXT]
    assert len(kat_records) > 20
    for r in kat_records:
        assert got[r] == want, (r, got[r][:20])
    # the seams were crossed: some KAT record starts less than 58 bytes before a multiple of 1 KiB
    starts = np.cumsum([0] + [len(t.encode()) for t in texts])[:-1]
    assert any((1024 - int(starts[r]) % 1024) < len(kat.KAT_TEXT) for r in kat_records)


@pytest.mark.parametrize("rng_mode", [0, 1])
def test_span_rows_on_the_kat_tokenizer_match_oracle(torch, native_lib, kat_tokenizer, rng_mode):
    import random
    rng = random.Random(5 + rng_mode)
    words = kat.KAT_TEXT.split()
    texts = [" ".join(kat.KAT_TEXT for _ in range(rng.randint(4, 40))) for _ in range(40)]
    texts += [" ".join(rng.choice(words) for _ in range(rng.randint(30, 400))) for _ in range(40)]
    S, B, seed = 512, 16, 99
    db = DeviceBatcher(task=native.SDL_TASK_SPAN, batch_size=B, sequence_length=S, seed=seed,
                       tokenizer=kat_tokenizer, rng_mode=rng_mode)
    ta, to, n = _arena(torch, texts)
    res = db.process(ta.data_ptr(), n, to.data_ptr(), len(texts))
    torch.cuda.synchronize()
    G = res.rows()
    ids, am, tt, lab = res.planes(G + (-G) % B)
    t5 = oracle_lib.T5Tok(kat_tokenizer)
    ob = oracle_lib.OracleBatcherEx(oracle_lib.Encoder("t5", t5), oracle_lib.SPAN, B, S, seed=seed,
                                    rng_mode=rng_mode)
    want = [r for r in (ob.push(t.encode()) for t in texts) if r is not None]
    while True:
        r = ob.flush()
        if r is None:
            break
        want.append(r)
    cat = {k: np.concatenate([w[k][:w["rows"]] for w in want]) for k in ("input_ids", "attention_mask", "labels")}
    assert G == cat["input_ids"].shape[0] > 0
    np.testing.assert_array_equal(ids[:G], cat["input_ids"])
    np.testing.assert_array_equal(am[:G], cat["attention_mask"])
    np.testing.assert_array_equal(lab[:G], cat["labels"])
    assert res.label_errors() == ob.span_errors()
