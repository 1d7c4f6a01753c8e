"""GPU parity of the grouped pending-word walk (tokenize_wordpiece.hip, state machine (b)):
a chunk's pending words -- first-probe misses -- are worked by G = 64 / pending lanes each
(8, 4, 2 or 1), so chunks are built here with 1..40 pending words, ASCII and accented,
short and up to the 16-byte fast-path limit, next to in-vocabulary filler, and every row is
checked against the oracle."""
import random

import numpy as np
import pytest

import oracle_lib  # noqa: F401  (the oracle_tok fixture)
from streaming_data_loader_amd.device import DeviceBatcher

from test_gpu_parity import framed_rows, run_device, torch  # noqa: F401

pytestmark = pytest.mark.gpu

LETTERS = "abcdefghijklmnopqrstuvwxyz"
ACCENTED = "éèçñöüåøæßàâêîôû"


def odd_word(rng, accented):
    n = rng.randint(3, 15)
    w = "".join(rng.choice(LETTERS) for _ in range(n))
    if accented:
        k = rng.randrange(len(w))
        w = w[:k] + rng.choice(ACCENTED) + w[k + 1:]
    return w


@pytest.mark.parametrize("pending", [1, 5, 8, 9, 16, 17, 33, 40])
def test_pending_groups_match_oracle(torch, native_lib, oracle_tok, pending):  # noqa: F811
    rng = random.Random(1000 + pending)
    filler = "the of and to in a is that for it as was with be by on not he".split()
    texts = []
    for rec in range(12):
        words = [odd_word(rng, rng.random() < 0.3) for _ in range(pending)]
        words += [rng.choice(filler) for _ in range(max(0, 150 - pending))]
        rng.shuffle(words)
        # ~1 KiB: one chunk holds about this record's words
        texts.append(" ".join(words)[:1000])
    db = DeviceBatcher(batch_size=16, sequence_length=512, mask_length=0, min_ids=0)
    ids = run_device(torch, db, texts).planes()[0]
    want = framed_rows(oracle_tok, texts, 512)
    assert ids.shape == want.shape
    bad = np.nonzero((ids != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} rows differ, first {bad[:5]}"
    db.close()
