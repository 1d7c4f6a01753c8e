"""The provider's JsonText filter: sdl_json_text_device
(json_text.hip) against the CPU oracle (oracle/json_text.py, a restatement of
provider_util.rs:60-64 create_json_text over tokio lines()).  CPU tests pin the
oracle with hand-written expectations; GPU tests are bit-exact on the records,
the line count and the invalid-line count, and run the records through the
Batcher (JSON lines in HBM -> batches without leaving the device)."""
import json
import os
import random
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import json_text as J  # noqa: E402

HAND = [  # (line, expected record | None | "invalid") -- serde_json semantics
    (b'{"text": "plain"}', b"plain"),
    (b'{"id": 7, "text": "a\\nb\\t\\"q\\"\\\\ \\/"}', b'a\nb\t"q"\\ /'),
    (b'{"text": "\\u00e9\\u4e2d\\ud83d\\ude00"}', "é中😀".encode()),
    (b'{"text": "raw \xc3\xa9 \xf0\x9f\x98\x80"}', "raw é 😀".encode()),
    (b'{"text": "first", "text": "last"}', b"last"),          # the map keeps the last
    (b'{"text": "s", "text": 5}', None),                      # last is not a string
    (b'{"te\\u0078t": "escaped key"}', b"escaped key"),
    (b'{"meta": {"text": "nested"}}', None),                  # not a top-level member
    (b'[{"text": "in array"}]', None),
    (b'"text"', None),
    (b'{"text": null}', None),
    (b'  {"text" : "ws" }  \r', b"ws"),
    (b'{"a": [1, -2.5e+3, true, false, null, {"b": []}], "text": "after"}', b"after"),
    (b'{}', None),
    (b'', "invalid"),                                         # empty line: EOF while parsing
    (b'{"text": "x",}', "invalid"),                           # trailing comma
    (b'{"text": "x"} {}', "invalid"),                         # trailing characters
    (b'{"text": "\\ud800"}', "invalid"),                      # lone leading surrogate
    (b'{"text": "\\udc00"}', "invalid"),                      # lone trailing surrogate
    (b'{"text": "a\tb"}', "invalid"),                         # raw control character
    (b'{"text": "\\x"}', "invalid"),                          # bad escape
    (b'{"text": "\xc3"}', "invalid"),                         # invalid UTF-8
    (b'{"n": 01}', "invalid"),
    (b'{"n": NaN}', "invalid"),
    (b'{"n": 1.}', "invalid"),
    (b'{"n": -}', "invalid"),
    (b'{"text": "unterminated}', "invalid"),
    (b'[' * 127 + b']' * 127, None),                          # 127 containers: serde's limit
    (b'[' * 128 + b']' * 128, "invalid"),
]


def test_oracle_hand_cases():
    for line, want in HAND:
        got = J.extract_line(line)
        if want == "invalid":
            assert got is J.INVALID, line
        else:
            assert got == want, line


def test_oracle_lines_like_tokio():
    assert J.split_lines(b"") == []
    assert J.split_lines(b"a\n") == [b"a"]
    assert J.split_lines(b"a\n\nb") == [b"a", b"", b"b"]
    assert J.split_lines(b"a\n\n") == [b"a", b""]


def fixture_jsonl(records, seed=0, n=None):
    """The fixture records as provider lines: json.dumps with varied key
    order, extra members, ASCII-escaped or raw UTF-8, plus hand cases."""
    rng = random.Random(seed)
    lines = []
    for i, t in enumerate(records if n is None else [records[rng.randrange(len(records))] for _ in range(n)]):
        obj = {"id": i, "title": f"t{i}", "text": t}
        if rng.random() < 0.3:
            obj = {"text": t, "meta": {"text": "no", "k": [1, 2.5, None]}, "id": i}
        lines.append(json.dumps(obj, ensure_ascii=rng.random() < 0.5).encode("utf-8"))
    return lines


def to_dev(torch, buf):
    a = np.zeros(len(buf) + 32, np.uint8)
    a[:len(buf)] = np.frombuffer(buf, np.uint8)
    return torch.from_numpy(a).cuda()


def device_records(torch, db, buf):
    d = to_dev(torch, buf)
    out = db.json_text(d.data_ptr(), len(buf))
    from streaming_data_loader_amd import native
    offs = np.zeros(out.n_records + 1, np.uint64)
    native.d2h(db._h, offs, out.d_offsets, offs.nbytes)
    text = np.zeros(int(out.text_bytes) + 16, np.uint8)
    native.d2h(db._h, text, out.d_text, text.nbytes)
    recs = [text[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(out.n_records)]
    assert (text[int(out.text_bytes):] == 0).all()
    return recs, out, d


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a HIP device"
    return t


@pytest.mark.gpu
def test_hand_cases_on_device(torch, native_lib):
    from streaming_data_loader_amd.device import DeviceBatcher
    db = DeviceBatcher(batch_size=8, sequence_length=128)
    buf = b"\n".join(line for line, _ in HAND) + b"\n"
    recs, out, _ = device_records(torch, db, buf)
    want, n_lines, n_bad = J.json_text(buf)
    assert recs == want
    assert (out.n_lines, out.n_invalid) == (n_lines, n_bad)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1])
def test_fixture_lines_and_noise(torch, native_lib, records, seed):
    """Fixture records as JSON lines mixed with the hand cases, random
    escapes and unicode, long lines, no trailing newline."""
    from streaming_data_loader_amd.device import DeviceBatcher
    rng = random.Random(seed)
    lines = fixture_jsonl(records, seed) + [line for line, _ in HAND]
    alphabet = ["a", " ", "é", "中", "😀", "\n", "\t", '"', "\\", "/", " ", "\x7f", "\u0001", "😀"]
    for i in range(300):
        t = "".join(rng.choice(alphabet) for _ in range(rng.choice([0, 1, 5, 40, 3000])))
        lines.append(json.dumps({"text": t, "i": i}, ensure_ascii=rng.random() < 0.5).encode("utf-8", "surrogatepass"))
    rng.shuffle(lines)
    buf = b"\n".join(lines)
    recs, out, _ = device_records(torch, db := DeviceBatcher(batch_size=8, sequence_length=128), buf)
    want, n_lines, n_bad = J.json_text(buf)
    assert (out.n_lines, out.n_invalid, out.n_records) == (n_lines, n_bad, len(want))
    assert recs == want
    db.close()


@pytest.mark.gpu
def test_dense_newlines_grow_the_line_list(torch, native_lib, records):
    """The newline list is sized for ~64-B lines; blank and tiny lines past that
    make the call grow it and write it again (one extra synchronisation).  Then
    a normal buffer on the same handle: the grown list is reused."""
    from streaming_data_loader_amd.device import DeviceBatcher
    db = DeviceBatcher(batch_size=8, sequence_length=128)
    rng = random.Random(11)
    lines = fixture_jsonl(records, 4)
    for i in range(30000):
        lines.append(rng.choice([b"", b"{}", b'{"text":""}', b'{"text":"a"}', b" ", b"1"]))
    rng.shuffle(lines)
    buf = b"\n".join(lines) + b"\n\n"
    assert buf.count(b"\n") > len(buf) // 64 + 4096
    recs, out, _ = device_records(torch, db, buf)
    want, n_lines, n_bad = J.json_text(buf)
    assert (out.n_lines, out.n_invalid, out.n_records) == (n_lines, n_bad, len(want))
    assert recs == want
    buf2 = b"\n".join(fixture_jsonl(records, 5))  # no trailing newline
    recs, out, _ = device_records(torch, db, buf2)
    want, n_lines, n_bad = J.json_text(buf2)
    assert (out.n_lines, out.n_records) == (n_lines, len(want)) and recs == want
    db.close()


@pytest.mark.gpu
def test_json_lines_to_batches_on_device(torch, native_lib, records, oracle_tok):
    """JSON lines in HBM -> JsonText -> Batcher (mlm S=128 B=8) without leaving
    the device: the same rows as the oracle Batcher over the extracted texts."""
    import oracle_lib
    from streaming_data_loader_amd.device import DeviceBatcher
    buf = b"\n".join(fixture_jsonl(records, 3)) + b"\n"
    db = DeviceBatcher(batch_size=8, sequence_length=128, seed=1234)
    recs, out, _d = device_records(torch, db, buf)
    res = db.process(out.d_text, int(out.text_bytes), out.d_offsets, int(out.n_records))
    torch.cuda.synchronize()
    got = res.planes()
    want = oracle_lib.oracle_rows(oracle_lib.Tok(), [r.decode("utf-8") for r in recs], 128, 19, 103, seed=1234, B=8)
    for j in range(4):
        np.testing.assert_array_equal(got[j], want[j])


def long_lines():
    """Lines >= 512 bytes (the wave-per-line kernels): every hand case padded
    with JSON whitespace, escape runs crossing 16-byte lanes and 1 KiB steps
    (chains of \\u escapes, backslash runs, surrogate pairs at every offset),
    and long invalid lines whose error sits deep inside."""
    pad = b" " * 600
    out = [(pad + line + b" \r", want) for line, want in HAND]
    out.append((b'{"text": "' + b"\\u00e9" * 500 + b'"}', "é".encode() * 500))
    out.append((b'{"text": "' + b"\\\\" * 700 + b'"}', b"\\" * 700))
    out.append((b'{"text": "' + b"\\ud83d\\ude00" * 200 + b'"}', "😀".encode() * 200))
    for k in range(0, 40):
        body = b"a" * (1000 + k) + b"\\ud83d\\ude00\\n\\\"" + b"b" * 30
        out.append((b'{"id": 1, "text": "' + body + b'"}', b"a" * (1000 + k) + "😀".encode() + b'\n"' + b"b" * 30))
    x = b"x" * 2000
    out += [
        (b'{"text": "' + x + b'\\q"}', "invalid"),                 # bad escape deep inside
        (b'{"text": "' + x, "invalid"),                             # unterminated
        (b'{"text": "' + x + b'\x01"}', "invalid"),                 # raw control character
        (b'{"text": "' + x + b'\xe2\x82"}', "invalid"),             # truncated UTF-8
        (b'{"text": "' + x + b'\xed\xa0\x80"}', "invalid"),         # UTF-8 surrogate
        (b'{"text": "' + x + b'\xc0\xaf"}', "invalid"),             # overlong
        (b'{"text": "' + x + b'\\udc00"}', "invalid"),              # lone trailing surrogate
        (b'{"text": "' + x + b'\\ud83d"}', "invalid"),              # lone leading surrogate
        (b'{"text": "' + x + b'"} x', "invalid"),                   # trailing characters
        (b'{"a": "' + x + b'", "n": 12}', None),                    # number ends the object
        (b'{"a": "' + x + b'", "n": 012}', "invalid"),
        (b'{"a": "' + x + b'", "text": tru}', "invalid"),
        (b'{"a": "' + x + b'", "text": true}', None),
        (b'{"a": "' + x + b'", "text": "' + x + b'", "text": "' + b"y" * 700 + b'"}', b"y" * 700),
        (b'{"te\\u0078t": "' + x + b'"}', x),                       # escaped key
        (b'{"meta": {"text": "' + x + b'"}}', None),
        (b'[' * 127 + b'"' + x + b'"' + b']' * 127, None),
        (b'[' * 128 + b'"' + x + b'"' + b']' * 128, "invalid"),
        (b'{"text": "' + "é".encode() * 1000 + b'", "n": -1.5e+7}', "é".encode() * 1000),
    ]
    return out


def test_oracle_long_cases():
    for line, want in long_lines():
        got = J.extract_line(line)
        if want == "invalid":
            assert got is J.INVALID, line[:80]
        else:
            assert got == want, line[:80]


@pytest.mark.gpu
def test_long_lines_on_device(torch, native_lib):
    """The wave-per-line parse and decode (lines >= 512 bytes) against the
    oracle, mixed with short lines so both kernels run in one call."""
    from streaming_data_loader_amd.device import DeviceBatcher
    db = DeviceBatcher(batch_size=8, sequence_length=128)
    lines = [line for line, _ in long_lines()] + [line for line, _ in HAND]
    random.Random(5).shuffle(lines)
    buf = b"\n".join(lines)
    recs, out, _ = device_records(torch, db, buf)
    want, n_lines, n_bad = J.json_text(buf)
    assert (out.n_lines, out.n_invalid, out.n_records) == (n_lines, n_bad, len(want))
    assert recs == want


@pytest.mark.gpu
@pytest.mark.parametrize("task,S,B,chunk", [("mlm", 128, 8, 20000), ("mlm", 512, 16, 65536), ("clm", 256, 4, 9000),
                                            ("span", 128, 8, 30000), ("mlm", 128, 8, 1 << 30)])
def test_json_to_frames_equals_one_call(torch, native_lib, records, task, S, B, chunk):
    """sdl_json_to_frames (chunks cut at line ends, rows carried across chunks,
    copies overlapped on three streams) hands the sink exactly the frames of
    one whole-buffer call: JsonText -> process -> pickle frames (flush)."""
    from streaming_data_loader_amd import native
    from streaming_data_loader_amd.device import DeviceBatcher
    kind = {"mlm": native.SDL_TASK_MLM, "clm": native.SDL_TASK_CLM, "span": native.SDL_TASK_SPAN}[task]
    tok = {"clm": native.GPT2_PROXY_TOKENIZER, "span": native.T5_PROXY_TOKENIZER}.get(task, native.BERT_PROXY_TOKENIZER)
    lines = fixture_jsonl(records, 7) * 3 + [line for line, _ in HAND] + [line for line, _ in long_lines()[:20]]
    random.Random(11).shuffle(lines)
    buf = b"\n".join(lines) + b"\n"
    db = DeviceBatcher(task=kind, batch_size=B, sequence_length=S, seed=42, tokenizer=tok)
    d = to_dev(torch, buf)
    jt = db.json_text(d.data_ptr(), len(buf))
    res = db.process(jt.d_text, int(jt.text_bytes), jt.d_offsets, int(jt.n_records))
    torch.cuda.synchronize()
    want = db.pickle_frames(res, res.rows(), True).frames()
    db2 = DeviceBatcher(task=kind, batch_size=B, sequence_length=S, seed=42, tokenizer=tok)
    got, st = db2.json_to_frames(buf, chunk_bytes=chunk)
    assert st.n_records == jt.n_records and st.n_invalid == jt.n_invalid and st.n_lines == jt.n_lines
    assert st.n_chunks >= (2 if chunk < len(buf) else 1)
    assert len(got) == len(want) and st.n_frames == len(want)
    for i, (a, b) in enumerate(zip(got, want)):
        assert a == b, f"frame {i} of {len(want)}"
