"""CPU model of tokenize_bpe.hip's bpe_lane (r05: one missed word per lane, <= 16 byte
symbols in registers) against tokenizers' BPE::merge_word (models/bpe/word.rs merge_all):
a min-heap of Merge {pos, rank, new_id} ordered by rank, then position, whose popped entry is
skipped when its symbol was merged away or the pair at its position no longer maps to its
new_id.  bpe_lane merges the lowest-rank pair, leftmost on ties, one merge per step, in a
compacted array, re-deriving only the two pairs a merge creates.  Both are run on random merge
tables (one rank per pair, as merges.txt lines; a pair repeated along a word ties on rank,
self-pairs like (a, a), chains of merges) and random words; the id sequences must be equal."""
import heapq
import random

import pytest


def merge_word_tokenizers(syms, merges):
    """word.rs merge_all (no dropout): symbols as a linked list, heap of (rank, pos, new_id)."""
    n = len(syms)
    c = list(syms)
    alive = [True] * n
    prev = list(range(-1, n - 1))
    nxt = list(range(1, n)) + [-1]
    heap = []
    for i in range(n - 1):
        m = merges.get((c[i], c[i + 1]))
        if m:
            heapq.heappush(heap, (m[0], i, m[1]))
    while heap:
        rank, pos, new_id = heapq.heappop(heap)
        if not alive[pos] or nxt[pos] == -1:
            continue
        np_ = nxt[pos]
        m = merges.get((c[pos], c[np_]))
        if not m or m[1] != new_id:
            continue
        c[pos] = new_id
        alive[np_] = False
        nxt[pos] = nxt[np_]
        if nxt[np_] != -1:
            prev[nxt[np_]] = pos
        if prev[pos] >= 0:
            p = prev[pos]
            m2 = merges.get((c[p], c[pos]))
            if m2:
                heapq.heappush(heap, (m2[0], p, m2[1]))
        if nxt[pos] != -1:
            m2 = merges.get((c[pos], c[nxt[pos]]))
            if m2:
                heapq.heappush(heap, (m2[0], pos, m2[1]))
    return [c[i] for i in range(n) if alive[i]]


def bpe_lane_model(syms, merges, LB=16):
    """The kernel's registers: s[LB], v[LB - 1] (rank << 16 | id, NOV = none), select-shift."""
    NOV = 0xFFFFFFFF

    def mv(a, b):
        m = merges.get((a, b))
        return NOV if m is None else (m[0] << 16 | m[1])

    n = len(syms)
    s = list(syms) + [0] * (LB - n)
    v = [mv(s[k], s[k + 1]) if k < n - 1 else NOV for k in range(LB - 1)]
    while True:
        br, bv, j = 0xFFFF, 0, -1
        for k in range(LB - 1):
            r = v[k] >> 16
            if r < br:
                br, bv, j = r, v[k], k
        if j < 0:
            break
        m = bv & 0xFFFF
        left = s[j - 1] if j >= 1 else 0
        right = s[j + 2] if j + 2 < LB else 0
        s = [s[k] if k < j else m if k == j else (s[k + 1] if k + 1 < LB else 0) for k in range(LB)]
        v = [v[k] if k < j - 1 else NOV if k <= j else (v[k + 1] if k + 1 < LB - 1 else NOV) for k in range(LB - 1)]
        n -= 1
        vl = mv(left, m) if j > 0 else NOV
        vr = mv(m, right) if j < n - 1 else NOV
        v = [vl if k == j - 1 else vr if k == j else v[k] for k in range(LB - 1)]
    return s[:n]


@pytest.mark.parametrize("seed", range(25))
def test_bpe_lane_equals_tokenizers_merge_order(seed):
    rng = random.Random(seed)
    alphabet = list(range(1, 7))  # few byte symbols: many repeated pairs
    merges = {}
    next_id = 100
    syms = list(alphabet)
    rank = 0
    for _ in range(rng.randint(5, 40)):  # merges over existing symbols (BPE training order)
        a, b = rng.choice(syms), rng.choice(syms)
        if (a, b) in merges:
            continue
        merges[(a, b)] = (rank, next_id)
        syms.append(next_id)
        next_id += 1
        rank += rng.choice([1, 1, 2])
    for _ in range(400):
        n = rng.randint(2, 16)
        word = [rng.choice(alphabet) for _ in range(n)]
        assert bpe_lane_model(word, merges) == merge_word_tokenizers(word, merges), (seed, word)
