"""CPU model of the Unigram chunk kernel's row DP (tokenize_unigram.hip, r05) against the
Viterbi it restates (unigram.hpp unigram_viterbi_masked: Unigram::encode_optimized's visit
order and strict-> replacement).

The kernel gives a Viterbi piece ("▁" + payload of L <= 16 bytes) a 16-lane DPP row: lane gl
holds node p = gl + 1 (after "▁" and p payload bytes) in registers; node 3 ("▁" alone) is the
"▁" piece or its unk.  Every candidate ending at p is read from the round's probe results up
front; the starts are visited in order (S, payload start 0, 1, ...), the base of payload start
i >= 1 being node i's score, broadcast by row_newbcast:(i - 1).  The unk relaxation of a start
whose one-char piece is missing is folded into that piece's slot.  This model runs exactly that
schedule (lane values updated step by step from a broadcast of the previous state) and checks
node scores, back pointers and the emitted ids against the sequential Viterbi on random
payloads with multi-byte chars, random candidate sets, tied scores and unk runs."""
import random
import struct

import pytest

NEG_INF = float("-inf")


def f32(x):
    return struct.unpack("<f", struct.pack("<f", x))[0]


def u8len_lead(b):
    return 1 if b < 0x80 else 2 if (b & 0xE0) == 0xC0 else 3 if (b & 0xF0) == 0xE0 else 4 if (b & 0xF8) == 0xF0 else 1


META = [0xE2, 0x96, 0x81]


def make_case(rng, L, Mm, Mf):
    """payload bytes (valid UTF-8, L bytes), candidate table {(s, e): (id, score)} over node
    positions of acc = "▁" + payload (s = 0 is the "▁" start, e/s >= 3 payload nodes)."""
    chars = []
    while sum(len(c) for c in chars) < L:
        room = L - sum(len(c) for c in chars)
        k = rng.choice([1, 1, 1, 2, 3, 4])
        k = min(k, room)
        if k == 1:
            chars.append(bytes([rng.randrange(0x61, 0x7B)]))
        elif k == 2:
            chars.append(chr(rng.randrange(0x80, 0x800)).encode())
        elif k == 3:
            chars.append(chr(rng.randrange(0x800, 0xD000)).encode())
        else:
            chars.append(chr(rng.randrange(0x10000, 0x10FFFF)).encode())
    payload = b"".join(chars)
    assert len(payload) == L
    acc = bytes(META) + payload
    n = L + 3
    bound = [True] * (n + 1)  # char boundaries of acc
    bound[1] = bound[2] = False
    for i in range(3, n):
        if (acc[i] & 0xC0) == 0x80:
            bound[i] = False
    cands = {}
    scores = [f32(-rng.choice([1.5, 2.0, 2.5, 3.0, 3.25, 4.0, 7.5])) for _ in range(6)]
    next_id = 4
    for s in [0] + list(range(3, n)):
        if not bound[s]:
            continue
        for e in range(s + 1, n + 1):
            if not bound[e]:
                continue
            if s == 0 and e - 3 > Mm:
                continue
            if s >= 3 and e - s > Mf:
                continue
            if s == 0 and e < 3:
                continue
            if rng.random() < 0.35:
                cands[(s, e)] = (next_id, rng.choice(scores) if rng.random() < 0.6 else f32(-rng.uniform(1, 9)))
                next_id += 1
    return acc, n, bound, cands


def viterbi_ref(acc, n, cands, unk_score, unk_id, maxlen):
    """unigram.hpp unigram_viterbi (nodes: score, start, id; -1 unset)."""
    score = [0.0] * (n + 1)
    start = [-1] * (n + 1)
    nid = [-1] * (n + 1)

    def relax(e, c, st, i):
        if start[e] < 0 or c > score[e]:
            score[e], start[e], nid[e] = c, st, i

    st = 0
    while st < n:
        mb = min(u8len_lead(acc[st]), n - st)
        base = score[st]
        single = False
        for e in range(st + 1, min(st + maxlen, n) + 1):
            if e < n and (acc[e] & 0xC0) == 0x80:
                continue
            c = cands.get((st, e))
            if c is None:
                continue
            relax(e, c[1] + base, st, c[0])
            if e - st == mb:
                single = True
        if not single:
            relax(st + mb, unk_score + base, st, unk_id)
        st += mb
    return score, start, nid


def backtrack(n, start, nid, cands, unk_id):
    """unigram.hpp unigram_backtrack (fused unk runs looked up whole)."""
    seq = []
    e = n
    while e > 0 and start[e] >= 0:
        seq.append((start[e], e, nid[e]))
        e = start[e]
    seq.reverse()
    out = []
    i = 0
    while i < len(seq):
        s, e, t = seq[i]
        if t == unk_id:
            j = i
            while j + 1 < len(seq) and seq[j + 1][2] == unk_id:
                j += 1
            whole = cands.get((s, seq[j][1]))
            out.append(whole[0] if whole else unk_id)
            i = j + 1
        else:
            out.append(t)
            i += 1
    return out


def row_dp_model(acc, n, cands, unk_score, unk_id, Mm, Mf):
    """The kernel's schedule: lanes gl = 0..15 hold node p = gl + 1 (acc node 3 + p)."""
    L = n - 3
    payload = acc[3:]
    # node 3: the "▁" piece (meta task 0) or its unk
    c3 = cands.get((0, 3))
    c3s, bp3 = (c3[1], (0, c3[0])) if c3 else (unk_score, (0, unk_id))
    best = [NEG_INF] * 16
    bp = [None] * 16
    lane_live = [gl + 1 <= L for gl in range(16)]
    bnd = [False] * 16
    qs = [0] * 16
    for gl in range(16):
        p = gl + 1
        if not lane_live[gl]:
            continue
        bnd[gl] = p == L or (payload[p] & 0xC0) != 0x80
        q = p - 1
        if bnd[gl]:
            while q > 0 and (payload[q] & 0xC0) == 0x80:
                q -= 1
        qs[gl] = q

    def cand_sc(gl, start_node, piece_ok, unk_ok):
        """score (or -inf) and id of the candidate (start_node, node 3 + p) from the round's
        results, the unk folded into a missing one-char piece's slot (the unk is no piece: the
        length bounds Mm / Mf do not apply to it)."""
        p = gl + 1
        c = cands.get((start_node, 3 + p)) if piece_ok else None
        if c is not None:
            return c[1], c[0]
        return (unk_score if unk_ok else NEG_INF), unk_id

    # start S: the meta piece "▁" + payload[0, p), base 0.0
    for gl in range(16):
        p = gl + 1
        if lane_live[gl] and p <= Mm:
            sc, i = cand_sc(gl, 0, True, False)
            best[gl] = sc + 0.0
            bp[gl] = (0, i) if best[gl] > NEG_INF else None
    # payload start 0 (node 3, base c3)
    for gl in range(16):
        p = gl + 1
        sc, i = cand_sc(gl, 3, lane_live[gl] and p <= Mf, bnd[gl] and qs[gl] == 0)
        c = sc + c3s
        if c > best[gl]:
            best[gl], bp[gl] = c, (3, i)
    # payload start i >= 1: base = row_newbcast:(i - 1) of the row's current values
    for i in range(1, 16):
        base = best[i - 1]  # (every lane reads the same snapshot; lane i-1 is final by now)
        new_best, new_bp = list(best), list(bp)
        for gl in range(16):
            p = gl + 1
            sc, tid = cand_sc(gl, 3 + i, lane_live[gl] and i < p and p - i <= Mf, bnd[gl] and qs[gl] == i)
            c = sc + base
            if c > best[gl]:
                new_best[gl], new_bp[gl] = c, (3 + i, tid)
        best, bp = new_best, new_bp
    score = [0.0] * (n + 1)
    start = [-1] * (n + 1)
    nid = [-1] * (n + 1)
    score[3], start[3], nid[3] = c3s, bp3[0], bp3[1]
    for gl in range(min(L, 16)):
        if bp[gl] is not None:
            score[4 + gl], start[4 + gl], nid[4 + gl] = best[gl], bp[gl][0], bp[gl][1]
    return score, start, nid


@pytest.mark.parametrize("seed", range(40))
def test_row_dp_equals_sequential_viterbi(seed):
    rng = random.Random(seed)
    unk_id = 2
    for _ in range(150):
        L = rng.randint(0, 16)
        Mm, Mf = rng.choice([(16, 16), (8, 12), (16, 6), (3, 3), (20, 17)])
        acc, n, bound, cands = make_case(rng, L, Mm, Mf)
        unk_score = f32(-rng.choice([10.0, 12.5, 3.0]))  # sometimes better than pieces
        maxlen = max([Mm + 3, Mf])
        ref_s, ref_st, ref_id = viterbi_ref(acc, n, cands, unk_score, unk_id, maxlen)
        got_s, got_st, got_id = row_dp_model(acc, n, cands, unk_score, unk_id, Mm, Mf)
        for e in range(3, n + 1):
            if not bound[e]:
                continue
            assert (got_s[e], got_st[e], got_id[e]) == (ref_s[e], ref_st[e], ref_id[e]), (seed, L, e)
        assert backtrack(n, got_st, got_id, cands, unk_id) == backtrack(n, ref_st, ref_id, cands, unk_id)
