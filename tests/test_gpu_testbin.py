"""The HIP path against the reference's own output, `data/test.bin` (see test_testbin_pin.py).

Two device runs over the dump's three texts with the WordPiece vocabulary the dump
determines (canonical pieces and one drawn alternate):
  * tokenizer ids per record (CLM rows, no length filter), against every non-wildcard id;
  * the reference's CPU config (`masking_cases.rs:13-21`: mlm, S=128, B=8) through
    `sdl_process_device`, masks undone through the labels, against the same ids in today's
    framing -- the pieces, the framing, the chunking and the mask/label planes together.
"""
import numpy as np
import pytest

from streaming_data_loader_amd import native
from streaming_data_loader_amd.device import DeviceBatcher
from test_testbin_pin import check_framed_rows, fixture, mismatches, record_runs, write_tokenizer

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a HIP device"
    return t


def _arena(torch, texts):
    blobs = [t.encode("utf-8") for t in texts]
    offs = np.zeros(len(blobs) + 1, np.uint64)
    np.cumsum([len(b) for b in blobs], out=offs[1:])
    arena = np.zeros(int(offs[-1]) + 16, np.uint8)
    arena[:int(offs[-1])] = np.frombuffer(b"".join(blobs), np.uint8)
    return torch.from_numpy(arena).cuda(), torch.from_numpy(offs.astype(np.int64)).cuda(), int(offs[-1])


@pytest.mark.parametrize("alt", [None, 0])
def test_device_ids_reproduce_dump(torch, native_lib, tmp_path, alt):
    meta = fixture()
    tok = write_tokenizer(meta, str(tmp_path), alt)
    S = 2048
    db = DeviceBatcher(task=native.SDL_TASK_CLM, batch_size=8, sequence_length=S, min_ids=0, tokenizer=tok)
    ta, to, n = _arena(torch, meta["texts"])
    res = db.process(ta.data_ptr(), n, to.data_ptr(), len(meta["texts"]))
    torch.cuda.synchronize()
    assert res.tokenize_errors() == 0
    ids, am, _, _ = res.planes()
    per = res.record_rows()
    g = 0
    for r, (want, complete, wild) in enumerate(record_runs(meta)):
        seq = []
        for _ in range(int(per[r])):
            z = int((am[g] == 0).sum())
            seq += ids[g, :S if z == 0 else z].tolist()
            g += 1
        assert seq[0] == 101 and seq[-2:] == [102, 102]
        got = seq[1:-2]  # strip encode_mask's extra [CLS] ... [SEP][SEP]
        assert not mismatches(got, want, complete, wild), (r, mismatches(got, want, complete, wild)[:5])


def test_reference_cpu_config_rows_reproduce_dump(torch, native_lib, tmp_path):
    meta = fixture()
    tok = write_tokenizer(meta, str(tmp_path))
    S, B = 128, 8
    db = DeviceBatcher(task=native.SDL_TASK_MLM, batch_size=B, sequence_length=S, seed=1234, tokenizer=tok)
    ta, to, n = _arena(torch, meta["texts"])
    res = db.process(ta.data_ptr(), n, to.data_ptr(), len(meta["texts"]))
    torch.cuda.synchronize()
    ids, am, tt, lab = res.planes()
    assert (tt == 0).all()
    assert int((lab != -100).sum()) > 0
    check_framed_rows(meta, ids, am, lab, S)
