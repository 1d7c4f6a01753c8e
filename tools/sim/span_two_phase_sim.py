"""CPU model of the two-phase span row kernels (pipeline.hip k_span_plan / k_span_write),
checked against the sequential T5Data::put_data loop the oracle restates
(oracle/orc_batcher.c ORC_SPAN, t5_data.rs:162-226) on arbitrary draw sequences.

Phase 1 (one lane per row): the pass recurrence with its plan entries
  {lp, gg, ip, sz} per pass, the pass count, the ids / labels ends and the error count;
  a row needing more than capr = LW // 2 + 2 passes is flagged (the device lists it for the
  one-pass kernel).
Phase 2 (one wave per row): marks at each pass's first ids / label position, a max-scan
  gives every position its pass, the value follows from the pass's entry.
"""
import random

EXTRA_BASE = 32000


def extra(k):
    return EXTRA_BASE + (k if k < 100 else 99)


def sequential(ids, n, S, LW, draws):
    """The oracle's loop: (input_ids row, labels row, errors)."""
    inp = [0] * S
    lab = [-100] * LW
    err = 0
    ip = lp = ap = 0
    p = 0
    while lp < S:
        g, sz = draws(p)
        g = min(g, S - lp, n - ip)
        for j in range(g):
            inp[lp + j] = ids[ip + j]
        lp += g
        ip += g
        sz = min(sz, S - lp, n - ip)
        if sz > 0:
            e = extra(p)
            err += p >= 100
            inp[lp] = e
            for i, v in [(ap, e)] + [(ap + j + 1, ids[ip + j]) for j in range(sz)]:
                if i < LW:
                    lab[i] = v
                else:
                    err += 1
            lp += 1
            ip += sz
            ap += sz + 1
        if n <= ip:
            err += p + 1 >= 100
            if ap < LW:
                lab[ap] = extra(p + 1)
            else:
                err += 1
            break
        p += 1
    return inp, lab, err


def plan(n, S, LW, draws, capr):
    """k_span_plan for one row: (entries, np, lp_end, ap_end, errors) or None (overflow)."""
    tab, Ip, Ap, bad = [], 0, 0, 0
    p = 0
    while True:
        gr, sr = draws(p)
        gs, ss = min(gr, n), min(sr, n)
        last = Ip + gs + ss >= n
        gg = min(gs, n - Ip) if last else gs
        sz = min(ss, n - Ip - gg) if last else ss
        lp, ap = Ip - Ap + p, Ap + p
        if p >= capr:
            return None
        tab.append((lp, gg, Ip, sz))
        if sz > 0:
            bad += p >= 100
            lo, hi = max(ap, LW), ap + sz + 1
            bad += max(hi - lo, 0)
        if last:
            bad += p + 1 >= 100
            bad += ap + (sz + 1 if sz > 0 else 0) >= LW
            return tab, p + 1, lp + gg + (1 if sz > 0 else 0), ap + (sz + 1 if sz > 0 else 0), bad
        Ip += gs + ss
        Ap += ss
        p += 1


def write(ids, S, LW, tab, np_, lp_end, ap_end):
    """k_span_write for one row: owner by max-scan over pass marks."""
    mk, mk2 = [0] * S, [0] * LW
    for p in range(np_):
        lp, gg, ip, sz = tab[p]
        ap = ip - lp + 2 * p
        if lp < S:
            mk[lp] = p
        if ap < LW:
            mk2[ap] = p
    inp, run = [], 0
    for q in range(S):
        if q < lp_end:
            run = max(run, mk[q])
            lp, gg, ip, sz = tab[run]
            off = q - lp
            inp.append(ids[ip + off] if off < gg else extra(run))
        else:
            inp.append(0)
    lab, run = [], 0
    ap_lim = min(ap_end, LW)
    for q in range(LW):
        if q < ap_lim:
            run = max(run, mk2[q])
            lp, gg, ip, sz = tab[run]
            off = q - (ip - lp + 2 * run)
            lab.append(extra(run) if off == 0 else ids[ip + gg + off - 1])
        else:
            lab.append(extra(np_) if q == ap_end else -100)
    return inp, lab


def run(trials=2000, seed=1):
    """Random rows and draw sequences; returns (checked, overflowed) counts."""
    rng = random.Random(seed)
    checked = overflow = 0
    for _ in range(trials):
        S = rng.choice([8, 16, 64, 128, 512])
        LW = max(S // 4, 1)
        n = rng.randint(1, S)
        ids = [rng.randint(1, 30000) for _ in range(n)]
        style = rng.random()
        seq = {}

        def draws(p):
            if p not in seq:
                if style < 0.3:
                    seq[p] = (rng.randint(0, 40), rng.randint(1, 5))  # default-like
                elif style < 0.6:
                    seq[p] = (rng.randint(0, 3), rng.randint(1, 2))   # tiny gaps: many passes
                elif style < 0.8:
                    seq[p] = (rng.randint(0, 3 * S), rng.randint(1, 3 * S))  # past the row
                else:
                    seq[p] = (rng.choice([0, 1, 16]), rng.choice([1, 1, 2, 9]))
            return seq[p]

        want = sequential(ids, n, S, LW, draws)
        pl = plan(n, S, LW, draws, LW // 2 + 2)
        if pl is None:
            overflow += 1
            assert want[2] > 0, "a row within the label width overflowed the plan"
            continue
        tab, np_, lp_end, ap_end, bad = pl
        got = write(ids, S, LW, tab, np_, lp_end, ap_end)
        assert got[0] == want[0], ("ids", S, n)
        assert got[1] == want[1], ("labels", S, n)
        assert bad == want[2], ("errors", bad, want[2])
        checked += 1
    return checked, overflow


if __name__ == "__main__":
    print(run())
