"""Full bench-size (256 MiB arena) checks for span (t5 Unigram) and clm (gpt2
byte-BPE), like test_gpu_parity.test_full_size_properties does for mlm, plus
the held-out corpus and 3000 generated strings through all three tokenizers
against `tokenizers`' own ids (tests/golden/heldout_ids.npz).

At 256 MiB the oracle cannot recompute everything, so the checks are
size-independent properties: every record's row count and the total id count
equal what the oracle gives for its text, no capacity flag is raised, and 24
seeded records' rows (global record index kept) are recomputed by the oracle
bit-exactly.  The held-out corpus (tests/golden/heldout_records.jsonl: text on
the image the proxy vocabularies were not trained on) is compared with the
goldens record for record."""
import json
import os

import numpy as np
import pytest

import oracle_lib
from streaming_data_loader_amd import native
from streaming_data_loader_amd.device import DeviceBatcher

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a HIP device"
    return t


def bench_arena(records, nbytes, seed=0x5D1B):
    import bench
    return bench.build_arena(records, nbytes, seed)


TASKS = {
    # task: (sdl task, tokenizer json, oracle encoder kind, oracle task, S, B)
    "span": (native.SDL_TASK_SPAN, native.T5_PROXY_TOKENIZER, "t5", oracle_lib.SPAN, 512, 256),
    "clm": (native.SDL_TASK_CLM, native.GPT2_PROXY_TOKENIZER, "gpt2", oracle_lib.CLM, 1024, 128),
}


def oracle_tok(kind):
    return oracle_lib.T5Tok() if kind == "t5" else oracle_lib.Gpt2Tok()


@pytest.mark.parametrize("task", sorted(TASKS))
def test_full_size_properties(torch, native_lib, records, task):
    sdl_task, tok_path, kind, otask, S, B_ = TASKS[task]
    tok = oracle_tok(kind)
    arena, offs, order = bench_arena(records, 256 << 20)
    ta = torch.from_numpy(arena).cuda()
    to = torch.from_numpy(offs.astype(np.int64)).cuda()
    db = DeviceBatcher(task=sdl_task, batch_size=B_, sequence_length=S, seed=1234, tokenizer=tok_path)
    N = len(arena) - 16
    res = db.process(ta.data_ptr(), N, to.data_ptr(), len(order))
    torch.cuda.synchronize()
    assert res.tokenize_errors() == 0
    assert res.label_errors() == 0
    # per record: ids and rows are fixed by its text (framing: gpt2 +2, t5 +2 around enc(..)+</s>)
    n_ids = np.array([len(tok.encode(r)) for r in records], np.int64)
    framed = n_ids + 2
    rows_of = np.where(framed >= 64, -(-framed // S), 0)
    got_rows = res.record_rows()
    np.testing.assert_array_equal(got_rows, rows_of[order])
    # tokenizer ids produced (t5: the template's </s> is produced by the tokenizer stage)
    tok_extra = 1 if kind == "t5" else 0  # the template's </s> is added with the framing
    assert res.tokens() == int((n_ids - tok_extra)[order].sum())
    G = res.rows()
    assert G == int(rows_of[order].sum())
    row_off = np.concatenate([[0], np.cumsum(got_rows)])
    enc = oracle_lib.Encoder(kind, tok)
    sample = [int(r) for r in np.random.default_rng(7).choice(len(order), 24, replace=False)]
    for r in sample:
        if got_rows[r] == 0:
            continue
        ob = oracle_lib.OracleBatcherEx(enc, otask, 4096, S, seed=1234)
        ob.set_next_record(r)
        assert ob.push(records[order[r]]) is None
        want = ob.flush()
        n = int(got_rows[r])
        assert want["rows"] == n
        a = int(row_off[r])
        ids, am, _, lab = res.planes(a + n)
        np.testing.assert_array_equal(ids[a:a + n], want["input_ids"][:n])
        np.testing.assert_array_equal(am[a:a + n], want["attention_mask"][:n])
        np.testing.assert_array_equal(lab[a:a + n], want["labels"][:n])


def heldout_records():
    with open(os.path.join(GOLDEN, "heldout_records.jsonl"), encoding="utf-8") as f:
        return [json.loads(l)["text"] for l in f]


def device_ids(torch, blobs, task, tok_path, S=2048):
    """Per-record tokenizer ids from CLM rows (no masking, no length filter)."""
    db = DeviceBatcher(task=native.SDL_TASK_CLM, batch_size=64, sequence_length=S, min_ids=0, tokenizer=tok_path)
    offs = np.zeros(len(blobs) + 1, np.uint64)
    np.cumsum([len(b) for b in blobs], out=offs[1:])
    arena = np.zeros(int(offs[-1]) + 16, np.uint8)
    arena[:int(offs[-1])] = np.frombuffer(b"".join(blobs), np.uint8)
    ta = torch.from_numpy(arena).cuda()
    to = torch.from_numpy(offs.astype(np.int64)).cuda()
    res = db.process(ta.data_ptr(), int(offs[-1]), to.data_ptr(), len(blobs))
    torch.cuda.synchronize()
    assert res.tokenize_errors() == 0
    ids, am, _, _ = res.planes()
    per = res.record_rows()
    out, g = [], 0
    for r in range(len(blobs)):
        seq = []
        for _ in range(int(per[r])):
            z = int((am[g] == 0).sum())
            seq += ids[g, :S if z == 0 else z].tolist()
            g += 1
        out.append(seq)
    return out


KINDS = {"bert": native.BERT_PROXY_TOKENIZER, "gpt2": native.GPT2_PROXY_TOKENIZER, "t5": native.T5_PROXY_TOKENIZER}


def framed(kind, ids):
    """encode_mask framing around tokenizer ids (the template's [CLS]/[SEP] and </s> are in `ids`)."""
    if kind == "bert":
        return [101] + list(ids) + [102, 102]
    eos = 50256 if kind == "gpt2" else 1
    return [eos] + list(ids) + [eos]


@pytest.mark.parametrize("kind", ["bert", "gpt2", "t5"])
def test_heldout_corpus_ids_match_tokenizers_goldens(torch, native_lib, kind):
    """The HIP path on the 3 MB held-out corpus against `tokenizers` itself
    (tests/golden/make_heldout_goldens.py: per-record id count + blake2b-64
    digest of Tokenizer.encode(text, True).ids)."""
    from test_heldout_goldens import digest_ids
    g = np.load(os.path.join(GOLDEN, "heldout_ids.npz"))
    recs = heldout_records()
    blobs = [r.encode("utf-8") for r in recs]
    got = device_ids(torch, blobs, kind, KINDS[kind])
    bad = []
    for i, seq in enumerate(got):
        ids = seq[1:-2] if kind == "bert" else seq[1:-1]  # strip the encode_mask framing
        if framed(kind, ids) != seq or len(ids) != int(g[f"{kind}_n"][i]) or digest_ids(ids) != int(g[f"{kind}_digest"][i]):
            bad.append(i)
    assert not bad, f"{len(bad)} of {len(blobs)} records differ, first {bad[:5]}: {recs[bad[0]][:80]!r}"


@pytest.mark.parametrize("kind", ["bert", "gpt2", "t5"])
def test_generated_strings_match_tokenizers_goldens(torch, native_lib, kind):
    """3000 seeded random-Unicode and long-identifier strings, id for id
    against `tokenizers` (tests/golden/heldout_ids.npz)."""
    g = np.load(os.path.join(GOLDEN, "heldout_ids.npz"))
    t, o = g["gen_text"], g["gen_off"]
    blobs = [t[o[i]:o[i + 1]].tobytes() for i in range(len(o) - 1)]
    got = device_ids(torch, blobs, kind, KINDS[kind])
    ids, off = g[f"{kind}_ids"], g[f"{kind}_off"]
    bad = [i for i in range(len(blobs)) if got[i] != framed(kind, ids[off[i]:off[i + 1]].tolist())]
    assert not bad, f"{len(bad)} of {len(blobs)} strings differ, e.g. {[blobs[i][:40] for i in bad[:3]]}"
