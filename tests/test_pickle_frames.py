"""Transport frames: every finished DataSet leaves the
reference as serde_pickle::to_vec(&dataset) (rust/src/transport/zmq_transmit.rs:71)
and the consumer reads it with pickle.loads (python/external_dataset.py:52).

CPU tests pin the oracle serializer (oracle/orc_pickle.c) to the consumer's
semantics: CPython's pickle.loads of every oracle frame equals the DataSet's
dict (field names and order of bert_data.rs:106-145, gpt_data.rs:53-62,
t5_data.rs:235-249; the BertData labels list has the filled rows only), for
all tasks, partial batches, >=1000-row and >=1000-wide lists (the APPENDS
batches) and negative labels.  Byte-exactness against the serde-pickle crate
itself is unpinned (no cargo here).  GPU tests check sdl_pickle_frames_device
byte-for-byte against the oracle on the device planes."""
import os
import pickle

import numpy as np
import pytest

import oracle_lib

TASKS = ("mlm", "clm", "span", "multi-label")


def planes(task, B, S, rows, seed=0):
    rng = np.random.default_rng(seed)
    LW = {"span": S // 4, "multi-label": 9}.get(task, S)
    ids = rng.integers(0, 60000, (B, S), dtype=np.int32)
    am = rng.integers(0, 2, (B, S), dtype=np.int32)
    tt = np.zeros((B, S), np.int32) if task in ("mlm", "multi-label") else None
    if task == "multi-label":
        lab = (rng.random((B, LW)) < 0.3).astype(np.float32)
    else:
        lab = rng.integers(-100, 60000, (B, LW), dtype=np.int32)
        lab[rng.random((B, LW)) < 0.5] = -100
    return LW, ids, am, tt, lab


def want_dict(task, rows, ids, am, tt, lab):
    """DataSet's Serialize view as the consumer sees it (python lists)."""
    d = {"input_ids": ids.tolist(), "attention_mask": am.tolist()}
    if task in ("mlm", "multi-label"):
        d["token_type_ids"] = tt.tolist()
        d["labels"] = [[float(x) for x in r] for r in lab[:rows]] if task == "multi-label" else lab[:rows].tolist()
    else:
        d["labels"] = lab.tolist()
    return d


@pytest.mark.parametrize("task,B,S,rows", [
    ("mlm", 4, 16, 4), ("mlm", 3, 12, 1), ("mlm", 2, 8, 0), ("clm", 3, 1024, 3), ("span", 2, 24, 1),
    ("multi-label", 5, 8, 5), ("multi-label", 1003, 4, 1001), ("mlm", 1000, 4, 1000), ("clm", 2, 2000, 2),
    ("span", 1, 4003, 1)])
def test_oracle_frame_loads_as_dataset(task, B, S, rows):
    LW, ids, am, tt, lab = planes(task, B, S, rows)
    frame = oracle_lib.pickle_dataset(task, B, S, LW, rows, ids, am, tt, lab)
    assert frame[:2] == b"\x80\x03" and frame[-1:] == b"."
    got = pickle.loads(frame)
    want = want_dict(task, rows, ids, am, tt, lab)
    assert list(got) == list(want)  # Serialize field order
    assert got == want


def test_oracle_frame_size_is_closed_form():
    # 5 bytes per int, "](" + "e" per list, "e(" per 1000 items: the layout the
    # device kernel computes without a scan
    B, S = 7, 1500
    LW, ids, am, tt, lab = planes("clm", B, S, B)
    frame = oracle_lib.pickle_dataset("clm", B, S, LW, B, ids, am, tt, lab)
    row = 3 + 5 * S + 2 * (S // 1000)
    plane = 3 + B * row
    keys = sum(5 + len(k) for k in ("input_ids", "attention_mask", "labels"))
    assert len(frame) == 4 + keys + 3 * plane + 2


# ---------------------------------------------------------------------------
# GPU: the device frames equal the oracle's, byte for byte
# ---------------------------------------------------------------------------
GPU_CASES = [("mlm", 8, 128), ("clm", 4, 1024), ("span", 8, 64), ("multi-label", 16, 32), ("multi-label", 1100, 8)]


@pytest.mark.gpu
@pytest.mark.parametrize("task,B,S", GPU_CASES)
@pytest.mark.parametrize("flush", [True, False])
def test_device_frames_match_oracle(native_lib, records, task, B, S, flush):
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from streaming_data_loader_amd import native
    from streaming_data_loader_amd.device import DeviceBatcher, arena_from_texts
    kind = {"mlm": native.SDL_TASK_MLM, "clm": native.SDL_TASK_CLM, "span": native.SDL_TASK_SPAN,
            "multi-label": native.SDL_TASK_MULTI_LABEL}[task]
    tok = {"clm": native.GPT2_PROXY_TOKENIZER, "span": native.T5_PROXY_TOKENIZER}.get(task,
                                                                                   native.BERT_PROXY_TOKENIZER)
    texts = list(records) * (30 if B > 1000 else 3)
    db = DeviceBatcher(task=kind, batch_size=B, sequence_length=S, seed=7, device=0, tokenizer=tok)
    arena, offs = arena_from_texts(texts)
    pad = np.zeros(len(arena) + 16, np.uint8)
    pad[:len(arena)] = arena
    ta = torch.from_numpy(pad).cuda()
    to = torch.from_numpy(offs.astype(np.int64)).cuda()
    if task == "multi-label":
        rng = np.random.default_rng(3)
        per = [rng.choice(9, size=rng.integers(0, 4), replace=False) for _ in texts]
        lo = np.zeros(len(texts) + 1, np.int64)
        np.cumsum([len(p) for p in per], out=lo[1:])
        tl = torch.from_numpy(np.concatenate(per).astype(np.int32)).cuda()
        tlo = torch.from_numpy(lo).cuda()
        res = db.process_labels(ta.data_ptr(), len(arena), to.data_ptr(), len(texts), tl.data_ptr(), tlo.data_ptr())
    else:
        res = db.process(ta.data_ptr(), len(arena), to.data_ptr(), len(texts))
    torch.cuda.synchronize()
    n = res.rows()
    assert n > B, "the case must span more than one batch"
    fr = db.pickle_frames(res, n, flush_partial=flush)
    torch.cuda.synchronize()
    nb = n // B + (1 if flush and n % B else 0)
    assert len(fr) == nb
    frames = fr.frames()
    ids, am, tt, lab = res.planes(nb * B)
    LW = lab.shape[1]
    for b, frame in enumerate(frames):
        rows = min(B, n - b * B)
        sl = slice(b * B, (b + 1) * B)
        want = oracle_lib.pickle_dataset(task, B, S, LW, rows, ids[sl], am[sl], None if tt is None else tt[sl],
                                         lab[sl])
        assert frame == want, f"{task} batch {b}: first diff at {_first_diff(frame, want)}"
    d = pickle.loads(frames[-1])
    assert d["input_ids"] == ids[(nb - 1) * B:nb * B].tolist()
    db.close()


def _first_diff(a, b):
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            return i
    return min(len(a), len(b))
