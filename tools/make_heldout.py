#!/usr/bin/env python3
"""Builds tests/golden/heldout_records.jsonl: English text already on the image
that was never used to train the proxy vocabularies or tune any table
(VERDICT r1 "bench and check on held-out text").  No network.

Sources (fixed order, deterministic on this image):
  1. CPython's pydoc_data.topics: each help topic is one record;
  2. docstrings of a fixed list of stdlib modules: one record per module
     (module docstring + every public class/function docstring, in name order);
  3. Perl's .pod manual pages under /usr/share/perl: one record per =head1
     section (POD markup lines dropped);
  4. /usr/share/doc/*/copyright license texts: one record per file.
Records are capped at 64 KiB (split on paragraph breaks) and the whole set at
--max-bytes, so the fixture stays small; bench.py tiles it like the fixture.

    python tools/make_heldout.py [--max-bytes 3000000]
"""
import argparse
import glob
import importlib
import inspect
import json
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "tests", "golden", "heldout_records.jsonl")

STDLIB = ["argparse", "asyncio", "collections", "concurrent.futures", "contextlib", "csv", "dataclasses", "datetime",
          "decimal", "difflib", "email", "enum", "fractions", "functools", "heapq", "http.client", "http.server",
          "inspect", "io", "itertools", "json", "logging", "mailbox", "multiprocessing", "os", "pathlib", "pickle",
          "random", "re", "shutil", "socket", "sqlite3", "ssl", "statistics", "string", "subprocess", "tarfile",
          "tempfile", "textwrap", "threading", "tkinter", "typing", "unittest", "urllib.request", "uuid", "xml.dom",
          "zipfile", "zoneinfo"]


def split_record(text, cap=64 << 10):
    """Records above `cap` bytes are split on paragraph breaks."""
    if len(text.encode("utf-8")) <= cap:
        return [text]
    out, cur = [], []
    size = 0
    for para in text.split("\n\n"):
        n = len(para.encode("utf-8")) + 2
        if cur and size + n > cap:
            out.append("\n\n".join(cur))
            cur, size = [], 0
        cur.append(para)
        size += n
    if cur:
        out.append("\n\n".join(cur))
    return out


def pydoc_topics():
    from pydoc_data import topics
    return [topics.topics[k] for k in sorted(topics.topics)]


def stdlib_docs():
    recs = []
    for name in STDLIB:
        try:
            mod = importlib.import_module(name)
        except Exception:
            continue
        parts = [inspect.getdoc(mod) or ""]
        for attr in sorted(dir(mod)):
            if attr.startswith("_"):
                continue
            obj = getattr(mod, attr, None)
            if inspect.isclass(obj) or inspect.isfunction(obj):
                d = inspect.getdoc(obj)
                if d and getattr(obj, "__module__", "").startswith(name.split(".")[0]):
                    parts.append(f"{attr}\n{d}")
        text = "\n\n".join(p for p in parts if p)
        if text:
            recs.append(text)
    return recs


def perl_pods():
    recs = []
    for f in sorted(glob.glob("/usr/share/perl/*/pod/*.pod") + glob.glob("/usr/share/perl/*/**/*.pod", recursive=True)):
        try:
            with open(f, encoding="utf-8", errors="replace") as fh:
                src = fh.read()
        except OSError:
            continue
        for sec in re.split(r"^=head1 ", src, flags=re.M)[1:]:
            lines = [l for l in sec.splitlines() if not l.startswith("=")]
            text = "\n".join(lines).strip()
            if text:
                recs.append(text)
    return recs


def copyrights():
    recs = []
    for f in sorted(glob.glob("/usr/share/doc/*/copyright")):
        try:
            with open(f, encoding="utf-8", errors="replace") as fh:
                recs.append(fh.read())
        except OSError:
            pass
    return recs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-bytes", type=int, default=3_000_000)
    args = ap.parse_args()
    seen, out, total = set(), [], 0
    for src in (pydoc_topics(), stdlib_docs(), perl_pods(), copyrights()):
        for text in src:
            for r in split_record(text):
                if r in seen:
                    continue
                seen.add(r)
                n = len(r.encode("utf-8"))
                if total + n > args.max_bytes:
                    continue
                out.append(r)
                total += n
    with open(OUT, "w", encoding="utf-8") as f:
        for r in out:
            f.write(json.dumps({"text": r}, ensure_ascii=False) + "\n")
    print(f"{len(out)} records, {total} bytes -> {os.path.relpath(OUT, REPO)}")


if __name__ == "__main__":
    main()
