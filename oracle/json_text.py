"""CPU oracle for the provider's JsonText filter -- TEST INFRASTRUCTURE ONLY
(imported by tests/, __graft_entry__.smoke() and bench.py's baseline leg; never
by the product path, which is json_text.hip behind sdl_json_text_device).

Restates what the reference's gzip/zstd providers do per inflated line
(gzip_file_provider.rs:30-50 -> SourceFilter::JsonText, source_filter.rs:15-20
-> provider_util.rs:60-64 create_json_text):

    let v: Value = serde_json::from_str(line.as_str()).unwrap();
    v[tag].as_str().map(|e| e.to_string())          // tag = "text"

over a buffer split into lines as tokio's `lines()` does.  serde_json (crate,
not vendored, not buildable here) is restated with Python's json plus the
points where serde_json is stricter: lone surrogate escapes, NaN/Infinity and
its recursion limit (128, i.e. at most 127 nested containers).  Numbers beyond
the f64 range (serde_json: an error) are accepted, as by the device path.
Parity is pinned by the hand-written expectations in tests/test_json_text.py;
against serde_json itself it is unpinned (no Rust toolchain here)."""
import json

INVALID = object()  # a line the reference's unwrap() panics on


def split_lines(buf):
    """tokio::io::AsyncBufReadExt::lines(): '\\n'-separated, an empty tail dropped."""
    parts = bytes(buf).split(b"\n")
    if parts and parts[-1] == b"":
        parts.pop()
    return parts


def _reject_constant(name):
    raise ValueError(f"{name} is not JSON")


def _depth_and_strings_ok(v, depth=0):
    if isinstance(v, (dict, list)):
        depth += 1
        if depth > 127:
            return False
        items = v.items() if isinstance(v, dict) else enumerate(v)
        for k, x in items:
            if isinstance(k, str) and not _utf8_ok(k):
                return False
            if not _depth_and_strings_ok(x, depth):
                return False
        return True
    if isinstance(v, str):
        return _utf8_ok(v)
    return True


def _utf8_ok(s):
    try:
        s.encode("utf-8")  # lone surrogates (from \\uD800-style escapes) fail here
        return True
    except UnicodeEncodeError:
        return False


def extract_line(line):
    """The record a line yields: bytes, None (valid, no string "text"), or INVALID."""
    try:
        s = bytes(line).decode("utf-8")
        v = json.loads(s, parse_constant=_reject_constant)
    except (UnicodeDecodeError, ValueError, RecursionError):
        return INVALID
    if not _depth_and_strings_ok(v):
        return INVALID
    if isinstance(v, dict) and isinstance(v.get("text"), str):
        return v["text"].encode("utf-8")
    return None


def json_text(buf):
    """(records, n_lines, n_invalid) for a buffer of JSON lines."""
    recs, bad = [], 0
    lines = split_lines(buf)
    for ln in lines:
        r = extract_line(ln)
        if r is INVALID:
            bad += 1
        elif r is not None:
            recs.append(r)
    return recs, len(lines), bad
