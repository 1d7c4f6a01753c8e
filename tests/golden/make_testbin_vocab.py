"""Reconstruct the bert-base-uncased sub-vocabulary behind the reference's `data/test.bin`.

Generation-time script (runs in the build container only; nothing on the GPU box reads
`/root/reference`). `data/test.bin` (4,312 B) is the only output of the reference's own
tokenizer path that the reference holds: an abomonation dump of `Vec<Vec<u32>>` -- a 24-B outer
header (ptr, len 8, cap 8), eight 24-B inner headers (ptr, len 128, cap 128) and 8 x 128 u32
ids of bert-base-uncased for the first records of `data/test.json.gz`.
The abomonation dependency that wrote it is commented out at `rust/Cargo.toml:25-26`, so no
code of the current reference produces it; the ids themselves are what `tokenizers` 0.13.1's
`Tokenizer::encode(text, true)` returned for bert-base-uncased
(`rust/src/tokenizer/tokenizer_holder.rs:19-28`).

What the dump determines: aligning its id runs with the fixture's BertNormalizer +
BertPreTokenizer words (run through `tokenizers` 0.22.2 here) gives every used id's piece
string (with `##` for continuation pieces). WordPiece is greedy longest-match-first, so over
ANY subset of the real vocabulary that contains every piece the real run chose, it chooses the
same pieces (a longer match in the subset would be a longer match in the full vocabulary).
A tokenizer.json holding exactly those pieces at their real indices (fillers elsewhere) must
therefore reproduce the reference's ids on these records -- which is what
`tests/test_testbin_pin.py` checks for the C oracle, `tokenizers` and the HIP path.

Framing of the dump (older than the reference's current `encode_mask`):
each record is `[CLS] ids [SEP]` (what the HF template alone adds; today's
`tokenizer_wrapper.rs:107-134` wraps that in one more `[CLS]` and two more `[SEP]`), cut into
rows of 128 with the tail zero-padded and no <64 filter; and in each record's third row the
first position holds 0 where the text has a piece (record 0: the `'` of "Bakiev's",
record 1: the `##cas` of "fracas"). Those two positions are kept as wildcards here.

Outputs (committed):
  tests/golden/testbin/tokenizer.json  -- BertNormalizer/BertPreTokenizer/WordPiece/BertProcessing,
                                          vocab of 30,522 (inferred pieces at real ids, fillers)
  tests/golden/testbin/vocab.txt
  tests/golden/testbin_rows.json       -- the decoded dump (data, 8 x 128 ids) + per-record runs
"""
from __future__ import annotations

import gzip
import json
import os
import re
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF_BIN = "/root/reference/data/test.bin"
VOCAB_SIZE = 30522
WILD = -1
SPECIAL = {0: "[PAD]", 100: "[UNK]", 101: "[CLS]", 102: "[SEP]", 103: "[MASK]"}


def decode_dump(raw: bytes) -> list[list[int]]:
    """abomonation `Vec<Vec<u32>>`: outer (ptr, len, cap), len inner (ptr, len, cap), then data."""
    _, n, _ = struct.unpack_from("<3Q", raw, 0)
    lens = [struct.unpack_from("<3Q", raw, 24 + 24 * i)[1] for i in range(n)]
    off = 24 + 24 * n
    rows = []
    for ln in lens:
        rows.append(list(struct.unpack_from("<%dI" % ln, raw, off)))
        off += 4 * ln
    assert off == len(raw), (off, len(raw))
    return rows


def record_runs(rows: list[list[int]]) -> list[dict]:
    """Rows -> per-record id runs: a record starts at a row beginning with [CLS]."""
    recs: list[list[int]] = []
    for row in rows:
        if row[0] == 101:
            recs.append([])
        recs[-1].extend(row)
    out = []
    for ids in recs:
        complete = 102 in ids
        if complete:
            end = ids.index(102) + 1
            assert all(v == 0 for v in ids[end:])
            ids = ids[:end]
        wild = [i for i, v in enumerate(ids) if v == 0]
        out.append({"ids": ids, "complete": complete, "wildcards": wild})
    return out


_ESC = re.compile(r"\\(u[0-9a-fA-F]{4}|.)")


def dump_texts() -> list[str]:
    """The `text` fields as the dump's (older) provider saw them.

    Aligning the dump with the fixture shows that every JSON `\\uXXXX` escape reached the
    tokenizer as its LAST hex digit alone: `\\u2190` (left arrow) -> "0" (id 1014 = "0"),
    `\\u2192` -> "2" (1016), `2006\\u00a0 U.S.` -> "20060 u.s." (2006 ##0), em dash + NBSP
    `\\u2014\\u00a0The` -> "40the" (40th ##e), `Lapp\\u00e9` -> "lapp9" (lap ##p ##9). Every
    other escape (`\\"`, `\\\\`, `\\n` ...) decodes as JSON does. Records are the lines that
    carry a `text` field, in file order (`provider_util.rs:60-64`).
    """
    out = []
    with gzip.open(os.path.join(HERE, "test.json.gz"), "rt", encoding="utf-8") as f:
        for line in f:
            line = _ESC.sub(lambda m: m.group(1)[-1] if m.group(1)[0] == "u" else m.group(0), line)
            obj = json.loads(line)
            if isinstance(obj.get("text"), str):
                out.append(obj["text"])
    return out


def words_of(text: str) -> list[str]:
    from tokenizers import normalizers, pre_tokenizers
    s = normalizers.BertNormalizer(lowercase=True).normalize_str(text)
    return [w for w, _ in pre_tokenizers.BertPreTokenizer().pre_tokenize_str(s)]


class Aligner:
    """Two phases.

    1. Word -> id-run alignment. The tokenizer is deterministic, so every occurrence of a word
       carries the same id run; a word seen before must match its run exactly, a new word takes
       k >= 1 ids (k = 1 tried first), a k = 1 word fixes its id's string. A wrong k is caught
       at the next known word, so the search stays shallow.
    2. Piece strings: each multi-piece word's split points, constrained by the ids whose
       strings are already fixed (k = 1 words, other words' pieces), propagated to a fixpoint;
       the rest must be unique or are reported.
    """

    def __init__(self):
        self.word_ids: dict[str, tuple] = {}
        self.id2s: dict[int, str] = {}
        self.s2id: dict[str, int] = {}
        self.role: dict[int, list] = {}  # id -> [uses as first piece, uses as continuation]

    def feasible(self, w: str, run: tuple) -> bool:
        """Some split of w into len(run) pieces agrees with every id whose string is known."""
        k = len(run)

        def rec(j: int, a: int) -> bool:
            if j == k:
                return a == len(w)
            x = run[j]
            s = self.id2s.get(x) if x not in (WILD, 100) else None
            if s is not None:
                body = s if j == 0 else (s[2:] if s.startswith("##") else None)
                if body is None or (j == 0 and s.startswith("##")):
                    return False
                return w.startswith(body, a) and rec(j + 1, a + len(body))
            return any(rec(j + 1, b) for b in range(a + 1, len(w) - (k - j - 1) + 1))
        return rec(0, 0)

    def _roles(self, run: tuple, sign: int) -> bool:
        ok = True
        for j, x in enumerate(run):
            if x in (WILD, 100):
                continue
            r = self.role.setdefault(x, [0, 0])
            r[0 if j == 0 else 1] += sign
            if r[0] and r[1]:
                ok = False
        return ok

    def align(self, recs: list[tuple[list[str], list[int], bool]]) -> list[list[tuple[int, int]]]:
        """Align all records in one search (a wrong choice in one record can show in a later one).

        recs: (words, ids without framing, complete). Returns per record (word index, #ids)."""
        sys.setrecursionlimit(200000)
        plans: list[list[tuple[int, int]]] = [[] for _ in recs]
        deepest = [0, 0, 0]

        def go(r: int, wi: int, ii: int) -> bool:
            if r == len(recs):
                return True
            words, ids, complete = recs[r]
            n = len(ids)
            if (r, ii) > tuple(deepest[:2]):
                deepest[:] = [r, ii, wi]
            if ii == n:
                if wi == len(words) or not complete:
                    return go(r + 1, 0, 0)
                return False
            if wi == len(words):
                return False
            plan = plans[r]
            w = words[wi]
            known = self.word_ids.get(w)
            if known is not None:
                k = len(known)
                run = tuple(ids[ii:ii + k])
                tail = not complete and ii + k > n
                ok = all(a == b or WILD in (a, b) for a, b in zip(run, known)) and (len(run) == k or tail)
                if not ok:
                    return False
                plan.append((wi, len(run)))
                if go(r, wi + 1, ii + len(run)):
                    return True
                plan.pop()
                return False
            for k in range(1, min(len(w), n - ii) + 1):
                run = tuple(ids[ii:ii + k])
                if 100 in run and k > 1:
                    continue
                if k == 1 and run[0] != WILD:
                    have = self.id2s.get(run[0])
                    if have is not None and have != w:
                        continue
                    if self.s2id.get(w, run[0]) != run[0]:
                        continue
                if not self.feasible(w, run):
                    continue
                if not self._roles(run, 1):
                    self._roles(run, -1)
                    continue
                self.word_ids[w] = run
                fixed = False
                if k == 1 and run[0] not in (WILD, 100) and run[0] not in self.id2s:
                    self.id2s[run[0]] = w
                    self.s2id[w] = run[0]
                    fixed = True
                plan.append((wi, k))
                if go(r, wi + 1, ii + k):
                    return True
                plan.pop()
                del self.word_ids[w]
                self._roles(run, -1)
                if fixed:
                    del self.id2s[run[0]]
                    del self.s2id[w]
            return False

        ok = go(0, 0, 0)
        if ok:
            # merge every occurrence's run (a wildcard in one is the real id in another);
            # wildcards left get a distinct pseudo id each, bound like any other id
            merged: dict[str, list] = {}
            for (words, ids, _), plan in zip(recs, plans):
                ii = 0
                for wi, k in plan:
                    run = ids[ii:ii + k]
                    ii += k
                    if len(run) != len(self.word_ids[words[wi]]):
                        continue  # a truncated tail
                    cur = merged.setdefault(words[wi], list(run))
                    for j, x in enumerate(run):
                        if cur[j] == WILD:
                            cur[j] = x
            pseudo = 0
            for w, cur in merged.items():
                for j, x in enumerate(cur):
                    if x == WILD:
                        pseudo += 1
                        cur[j] = -1000 - pseudo
                self.word_ids[w] = tuple(cur)
                if len(cur) == 1 and cur[0] not in self.id2s and cur[0] != 100:
                    if self.s2id.get(w, cur[0]) == cur[0]:
                        self.id2s[cur[0]] = w
                        self.s2id[w] = cur[0]
        if not ok:
            r, ii, wi = deepest
            words, ids, _ = recs[r]
            raise RuntimeError("no alignment; deepest: record %d words %r ids %r" % (
                r, words[max(0, wi - 4):wi + 4], ids[max(0, ii - 4):ii + 6]))
        return plans

    def split_domains(self) -> dict[str, tuple[tuple, list]]:
        """Phase 2: the admissible split points of every multi-piece word.

        Constraint propagation to a fixpoint: a split must agree with every id whose string is
        known, and an id on which all of a word's remaining splits agree becomes known.
        Returns word -> (id run, remaining splits)."""
        multi = {w: r for w, r in self.word_ids.items() if len(r) > 1 and 100 not in r}
        cands: dict[str, list] = {}
        for w, run in multi.items():
            k = len(run)
            out = []

            def rec(a, j, acc):
                if j == k:
                    if a == len(w):
                        out.append(tuple(acc))
                    return
                for b in range(a + 1, len(w) - (k - j - 1) + 1):
                    acc.append(w[a:b] if j == 0 else "##" + w[a:b])
                    rec(b, j + 1, acc)
                    acc.pop()
            rec(0, 0, [])
            cands[w] = [c for c in out if all(layout_ok(x, p) for x, p in zip(run, c))]
        changed = True
        while changed:
            changed = False
            for w, run in multi.items():
                keep = [c for c in cands[w]
                        if all(self.id2s.get(x, p) == p and self.s2id.get(p, x) == x
                               for x, p in zip(run, c))]
                if not keep:
                    raise RuntimeError("no split for %r %r" % (w, run))
                if len(keep) != len(cands[w]):
                    cands[w] = keep
                    changed = True
                for j, x in enumerate(run):
                    vals = {c[j] for c in keep}
                    if len(vals) == 1 and x not in self.id2s:
                        p = vals.pop()
                        if self.s2id.get(p, x) != x:
                            raise RuntimeError("conflict on %r" % p)
                        self.id2s[x] = p
                        self.s2id[p] = x
                        changed = True
        return {w: (multi[w], cands[w]) for w in multi if len(cands[w]) > 1}

    def assignments(self, domains, check, rng=None, limit=1):
        """Yield up to `limit` id->string completions of the ambiguous words that are globally
        consistent and pass `check(id2s)` (every word re-tokenizes to its run). Forward
        checking: every choice filters the other words' splits before the search goes on."""
        found = [0]

        def consistent(run, c, b2s, s2b):
            for x, p in zip(run, c):
                have = b2s.get(x)
                if have is not None and have != p:
                    return False
                if s2b.get(p, x) != x:
                    return False
            return True

        def rec(doms, b2s, s2b):
            if found[0] >= limit:
                return
            if not doms:
                if check(b2s):
                    found[0] += 1
                    yield dict(b2s)
                return
            w = min(doms, key=lambda v: (len(doms[v][1]), v))
            run, cs = doms[w]
            cs = list(cs)
            if rng is not None:
                rng.shuffle(cs)
            else:
                # canonical: the most balanced split (least sum of squared piece lengths)
                cs.sort(key=lambda c: (sum(len(p.lstrip("#")) ** 2 for p in c), [-len(p) for p in c]))
            for c in cs:
                nb, ns = dict(b2s), dict(s2b)
                for x, p in zip(run, c):
                    nb[x] = p
                    ns[p] = x
                rest = {}
                for v, (rv, cv) in doms.items():
                    if v == w:
                        continue
                    keep = [d for d in cv if consistent(rv, d, nb, ns)]
                    if not keep:
                        break
                    rest[v] = (rv, keep)
                else:
                    yield from rec(rest, nb, ns)
                if found[0] >= limit:
                    return
        yield from rec(dict(domains), dict(self.id2s), dict(self.s2id))


def layout_ok(x: int, p: str) -> bool:
    """bert-base-uncased's layout: ids 999..1995 are the single (non-`##`) characters; no id
    from 1996 on is one (the dump agrees: digits at 1014-1023, `:` 1024, `[` 1031, `a` 1037)."""
    if x < 0:
        return True
    single = len(p) == 1
    return single if 999 <= x <= 1995 else not single


def greedy(w: str, vocab: dict[str, int]) -> list[int]:
    out, a = [], 0
    if len(w) > 100:
        return [100]
    while a < len(w):
        for b in range(len(w), a, -1):
            s = w[a:b] if a == 0 else "##" + w[a:b]
            if s in vocab:
                out.append(vocab[s])
                a = b
                break
        else:
            return [100]
    return out


def main() -> None:
    raw = open(REF_BIN, "rb").read()
    rows = decode_dump(raw)
    runs = record_runs(rows)
    texts = dump_texts()
    al = Aligner()
    recs = []
    for r, run in enumerate(runs):
        ids = run["ids"]
        assert ids[0] == 101
        inner = ids[1:-1] if run["complete"] else ids[1:]
        recs.append((words_of(texts[r]), [WILD if v == 0 else v for v in inner], run["complete"]))
    plans = al.align(recs)
    for r, run in enumerate(runs):
        words, inner, _ = recs[r]
        plan = plans[r]
        run["words_consumed"] = len(plan)
        if not run["complete"]:
            # the run may end inside its last word: keep nothing that word alone implied
            wi, k = plan[-1]
            w = words[wi]
            if sum(1 for j, _ in plan if words[j] == w) == 1 and w in al.word_ids:
                rr = al.word_ids.pop(w)
                if len(rr) == 1 and al.id2s.get(rr[0]) == w:
                    del al.id2s[rr[0]]
                    del al.s2id[w]
        print(f"record {r}: {len(inner)} ids over {len(plan)} of {len(words)} words")
    domains = al.split_domains()
    print("words whose split the dump leaves open:", sorted(domains))
    all_words = [(recs[r][0], runs[r]) for r in range(len(runs))]

    def reproduces(id2s: dict[int, str]) -> bool:
        vocab = {p: x for x, p in id2s.items()}
        for x, p in SPECIAL.items():
            vocab[p] = x
        for words, run in all_words:
            got = []
            for w in words:
                got.extend(greedy(w, vocab))
                if len(got) >= len(run["ids"]):
                    break
            inner = run["ids"][1:-1] if run["complete"] else run["ids"][1:]
            if run["complete"] and len(got) != len(inner):
                return False
            if any(v != 0 and g != v for g, v in zip(got, inner)):
                return False
        return True

    canon = next(al.assignments(domains, reproduces), None)
    if canon is None:
        raise RuntimeError("no admissible vocabulary")
    import random
    alts = list(al.assignments(domains, reproduces, rng=random.Random(0x5D1B), limit=4))
    open_ids = sorted({x for w in domains for x in domains[w][0]} - set(al.id2s))
    # a wildcard's piece (the dump holds 0 there) goes to a placeholder id the dump never uses
    placeholder = {}
    for x in sorted(canon, reverse=True):
        if x < 0:
            placeholder[x] = VOCAB_SIZE - 1 - len(placeholder)
    real_open = [x for x in open_ids if x >= 0]
    print(f"{len([x for x in canon if x >= 0])} pieces at real ids; {len(real_open)} ids with an "
          f"open string; {len(placeholder)} wildcard pieces; {len(alts)} alternates")

    def remap(sol):
        return {str(placeholder.get(x, x)): p for x, p in sorted(sol.items())}

    for r, run in enumerate(runs):
        vocab = {p: placeholder.get(x, x) for x, p in canon.items()}
        got = []
        for w in recs[r][0]:
            got.extend(greedy(w, vocab))
        run["wildcard_ids_here"] = [got[i - 1] for i in run["wildcards"]]
    meta = {
        "source": "reference data/test.bin: abomonation Vec<Vec<u32>> [8,128] of bert-base-uncased "
                  "ids (tokenizers 0.13.1), decoded by tests/golden/make_testbin_vocab.py",
        "rows": rows,
        "texts": texts[:len(runs)],
        "records": [{k: v for k, v in run.items() if k != "ids"} for run in runs],
        "vocab_size": VOCAB_SIZE,
        "pieces": remap(canon),
        "placeholder_ids": sorted(placeholder.values()),
        "open_ids": real_open,
        "alternates": [{str(placeholder.get(x, x)): a[x] for x in real_open + sorted(placeholder)}
                       for a in alts],
    }
    with open(os.path.join(HERE, "testbin_rows.json"), "w", encoding="utf-8") as f:
        json.dump(meta, f, ensure_ascii=False, separators=(",", ":"))
    print("wrote testbin_rows.json")


if __name__ == "__main__":
    main()
