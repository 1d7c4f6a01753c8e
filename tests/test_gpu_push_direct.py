"""Small calls on the host path (sdl_batcher_push / push_many of a few records).

They take two shortcuts the large path does not: one workgroup runs the chunk scan,
compaction, record framing, row scan and row map (k_downstream_small), and the rows go
straight into the back batch and a pre-allocated next one in the same pass
(k_rows_direct), rows past those two batches through the segment copy.  Checked here
against the C oracle where a record's rows overrun the two batches many times over
(S=16, B=1..3), for every tokenizer; and the reference's panic when a record arrives
after get_working_batch emptied the store (gen_batcher.rs:45, store.back_mut().unwrap())."""
import numpy as np
import pytest

import oracle_lib
from streaming_data_loader_amd import batcher as Bt
from streaming_data_loader_amd import native

pytestmark = pytest.mark.gpu


def drain(gt, texts):
    got = []
    for t in texts:
        d = gt.create_sync_batch(t)
        if d is not None:
            got.append(d)
    while True:
        d = gt.get_working_batch()
        if d is None or not d.rows:
            break
        got.append(d)
    return got


def planes(batches):
    keys = ("input_ids", "attention_mask", "token_type_ids", "labels")
    return [np.concatenate([np.asarray(getattr(d, k))[:d.rows] for d in batches]) for k in keys]


@pytest.mark.parametrize("B", [1, 2, 3])
def test_per_record_rows_past_the_direct_window_match_oracle(native_lib, records, B):
    texts = records[:10]
    S, k, seed = 16, 2, 77
    gt = Bt.GenTokenizer(Bt.ModelType.Bert, Bt.BatchConfig(B, S), Bt.Mask(k, 103), Bt.TokenizerConfig(),
                         chunk=True, seed=seed)
    got = planes(drain(gt, texts))
    want = oracle_lib.oracle_rows(oracle_lib.Tok(), texts, S, k, seed=seed, B=B)
    assert got[0].shape[0] > 3 * B * len(texts)  # most rows went through the segment copy
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)


@pytest.mark.parametrize("task", [Bt.TaskType.Clm, Bt.TaskType.Span])
def test_per_record_equals_one_call_other_tokenizers(native_lib, records, task):
    """byte-BPE (clm) and Unigram (span) through the small-call kernels, per record, equal
    one push_many of the same records (> 1 MiB: the large path)."""
    texts = [records[i % len(records)] for i in range(700)]
    assert sum(len(t.encode()) for t in texts) > (1 << 20)
    S, B = (128, 4)
    a = Bt.GenTokenizer.from_config(Bt.get_case(task, False, S, B, 1234))
    per = drain(a, texts)
    b = Bt.GenTokenizer.from_config(Bt.get_case(task, False, S, B, 1234))
    one = b.create_sync_batches(texts)
    while True:
        d = b.get_working_batch()
        if d is None or not d.rows:
            break
        one.append(d)
    keys = ("input_ids", "attention_mask", "labels")
    for key in keys:
        x = np.concatenate([np.asarray(getattr(d, key))[:d.rows] for d in per])
        y = np.concatenate([np.asarray(getattr(d, key))[:d.rows] for d in one])
        np.testing.assert_array_equal(x, y)


def test_record_after_the_store_is_emptied_fails_like_the_reference(native_lib, records):
    gt = Bt.GenTokenizer(Bt.ModelType.Bert, Bt.BatchConfig(2, 128), Bt.Mask(19, 103), Bt.TokenizerConfig(),
                         chunk=True, seed=1)
    drain(gt, records[:3])
    assert gt.get_working_batch() is None
    # fewer than 64 ids: the reference returns None before touching the store
    assert gt.create_sync_batch("a short record") is None
    with pytest.raises(native.SDLError, match="store"):
        gt.create_sync_batch(records[0])


@pytest.mark.parametrize("model", [Bt.ModelType.Bert, Bt.ModelType.Gpt2])
def test_unigram_capacity_flag_on_the_fused_small_push(native_lib, records, model, monkeypatch):
    """mlm / clm on the t5 tokenizer take the fused small push (k_rows writes the host
    batches, k_downstream_small the status words): a Unigram capacity overflow must still
    fail the call, as it does on the direct and large paths.  SDL_UNI_ITEM_CAP clamps the
    long-item list so a record with a few long items (words past the 48 bytes a Viterbi job
    takes) overflows it."""
    monkeypatch.setenv("SDL_UNI_ITEM_CAP", "1")
    gt = Bt.GenTokenizer(model, Bt.BatchConfig(4, 128), Bt.Mask(19, 103) if model == Bt.ModelType.Bert else
                         Bt.Gpt(), Bt.TokenizerConfig(native.T5_PROXY_TOKENIZER), chunk=True, seed=3)
    long_words = " ".join(["internationalization" * 3, "characteristically" * 3, "uncharacteristically" * 3])
    with pytest.raises(native.SDLError, match="capacity"):
        gt.create_sync_batch(records[0] + " " + long_words)


def test_unigram_small_push_without_overflow_raises_nothing(native_lib, records):
    """The same pairing without the clamp: long words are items, no error word is set."""
    gt = Bt.GenTokenizer(Bt.ModelType.Bert, Bt.BatchConfig(4, 128), Bt.Mask(19, 103),
                         Bt.TokenizerConfig(native.T5_PROXY_TOKENIZER), chunk=True, seed=3)
    for t in records[:8]:
        gt.create_sync_batch(t + " internationalization characteristically")


def test_short_calls_after_long_ones_read_no_stale_status(native_lib, records):
    """The mapped status words (row offsets, label and tokenizer error words) are rewritten
    by every call: push_many of many records, then single records, then a few, equal the
    per-record sequence row for row and raise nothing."""
    S, B, seed = 128, 4, 21
    seq = [records[:40], records[40:41], records[41:44], records[44:45], records[45:50]]
    a = Bt.GenTokenizer(Bt.ModelType.Bert, Bt.BatchConfig(B, S), Bt.Mask(19, 103), Bt.TokenizerConfig(),
                        chunk=True, seed=seed)
    mixed = []
    for part in seq:
        if len(part) == 1:
            d = a.create_sync_batch(part[0])
            mixed += [d] if d is not None else []
        else:
            mixed += a.create_sync_batches(part)
    while True:
        d = a.get_working_batch()
        if d is None or not d.rows:
            break
        mixed.append(d)
    b = Bt.GenTokenizer(Bt.ModelType.Bert, Bt.BatchConfig(B, S), Bt.Mask(19, 103), Bt.TokenizerConfig(),
                        chunk=True, seed=seed)
    per = drain(b, records[:50])
    for g, w in zip(planes(mixed), planes(per)):
        np.testing.assert_array_equal(g, w)


@pytest.mark.parametrize("B", [1, 4])
def test_per_record_rng_mode_1_matches_oracle(native_lib, records, B):
    """rng_mode 1 on the per-record push: nothing is walked beside the tokenizer on the small
    path, so k_rows' first pass skips every row and its late pass walks them all, writing them
    straight into the host batches (rows past the two batches through the segment copy)."""
    texts = records[:12]
    S, k, seed = 64, 9, 31
    gt = Bt.GenTokenizer(Bt.ModelType.Bert, Bt.BatchConfig(B, S), Bt.Mask(k, 103), Bt.TokenizerConfig(),
                         chunk=True, seed=seed, rng_mode=1)
    got = planes(drain(gt, texts))
    want = oracle_lib.oracle_rows(oracle_lib.Tok(), texts, S, k, seed=seed, B=B, rng_mode=1)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)
