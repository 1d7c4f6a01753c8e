"""The provider's gzip inflate: sdl_gzip_inflate_device
(inflate.hip, one wave per member) against the CPU oracle (oracle/orc_inflate.c,
an RFC 1951/1952 restatement with zlib's error rules), which is pinned here
against CPython's zlib on streams of every block type, every gzip header field,
and the reference's own data/test.json.gz (tests/golden/test.json.gz).  Member
outputs must be bit-exact; corrupt members must fail (the reference's
`next_line().await.unwrap()` panics) with the oracle's reason where the reason
is well defined."""
import gzip
import json
import os
import random
import struct
import zlib

import numpy as np
import pytest

import oracle_lib

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF_GZ = os.path.join(GOLDEN, "test.json.gz")

STRATEGIES = [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FIXED]


def gz_member(data, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, flags=0, extra=b"", name=b"", comment=b"",
              mem_level=8, flush_every=0):
    """One gzip member with the given header fields around zlib's raw DEFLATE."""
    co = zlib.compressobj(level, zlib.DEFLATED, -15, mem_level, strategy)
    if flush_every:
        body = b"".join(co.compress(data[i:i + flush_every]) + co.flush(zlib.Z_FULL_FLUSH)
                        for i in range(0, len(data), flush_every)) + co.flush()
    else:
        body = co.compress(data) + co.flush()
    flg = flags
    hdr = bytearray(b"\x1f\x8b\x08\x00" + struct.pack("<I", 0) + b"\x00\xff")
    if extra:
        flg |= 4
        hdr += struct.pack("<H", len(extra)) + extra
    if name:
        flg |= 8
        hdr += name + b"\x00"
    if comment:
        flg |= 16
        hdr += comment + b"\x00"
    hdr[3] = flg
    if flg & 2:
        hdr += struct.pack("<H", zlib.crc32(bytes(hdr)) & 0xFFFF)
    return bytes(hdr) + body + struct.pack("<II", zlib.crc32(data), len(data) & 0xFFFFFFFF)


def bgzf(data, block=65280, level=6):
    """BGZF (bgzip's layout): members of <= `block` input bytes, each with the
    'BC' extra subfield holding its size - 1, then the empty EOF member."""
    out = []
    for i in range(0, len(data), block):
        m = gz_member(data[i:i + block], level, extra=b"BC\x02\x00\x00\x00")
        m = bytearray(m)
        m[16:18] = struct.pack("<H", len(m) - 1)
        out.append(bytes(m))
    eof = bytearray(gz_member(b"", 6, extra=b"BC\x02\x00\x00\x00"))
    eof[16:18] = struct.pack("<H", len(eof) - 1)
    return b"".join(out) + bytes(eof)


def payloads(records):
    rng = random.Random(7)
    lines = "".join(json.dumps({"id": i, "text": t}) + "\n" for i, t in enumerate(records)).encode()
    return {
        "empty": b"",
        "one": b"x",
        "jsonl": lines,
        "jsonl_x3": lines * 3,
        "random": bytes(rng.randrange(256) for _ in range(70000)),  # stored blocks
        "run": b"a" * 100000,                                          # distance-1 copies
        "period": (b"abcdefghij" * 9000)[:90000],
        "mixed": lines[:20000] + bytes(rng.randrange(256) for _ in range(3000)) + b"z" * 5000 + lines[20000:60000],
    }


def corpus(records):
    """(name, member bytes, expected inflated bytes)"""
    out = []
    for pname, data in payloads(records).items():
        for level in (0, 1, 6, 9):
            for st in STRATEGIES:
                if level == 0 and st != zlib.Z_DEFAULT_STRATEGY:
                    continue
                out.append((f"{pname}/l{level}/s{st}", gz_member(data, level, st), data))
    data = payloads(records)["jsonl"]
    out.append(("header fields", gz_member(data, extra=b"ab\x03\x00xyz", name=b"file.json", comment=b"c",
                                           flags=2), data))
    out.append(("full flushes", gz_member(data, flush_every=4096), data))
    out.append(("memlevel 1", gz_member(data, 9, mem_level=1), data))
    out.append(("gzip module", gzip.compress(data, 9), data))
    return out


def corrupt_cases(records):
    """(name, member bytes, expected status) -- reasons that do not depend on
    where a decoder notices the damage"""
    data = payloads(records)["jsonl"][:30000]
    good = gz_member(data)
    bad_crc = bytearray(good)
    bad_crc[-8] ^= 1
    bad_size = bytearray(good)
    bad_size[-4] ^= 1
    bad_magic = bytearray(good)
    bad_magic[1] = 0x8c
    reserved = bytearray(good)
    reserved[3] |= 0x20
    hcrc = bytearray(gz_member(data, flags=2))
    hcrc[10] ^= 1
    btype3 = bytearray(gz_member(b"hello"))
    btype3[10] = 0x07  # BFINAL 1, BTYPE 3
    stored = bytearray(gz_member(b"hello world", level=0))
    stored[13] ^= 0xFF  # NLEN
    far = gz_member(b"")[:10] + bytes([0x03, 0x02]) + gz_member(b"")[12:]  # fixed block: match before any output
    return [
        ("crc", bytes(bad_crc), 13),
        ("isize", bytes(bad_size), 11),
        ("magic", bytes(bad_magic), 3),
        ("reserved flag", bytes(reserved), 3),
        ("header crc", bytes(hcrc), 4),
        ("btype 3", bytes(btype3), 5),
        ("stored nlen", bytes(stored), 6),
        # zlib (and, with multiple_members off, the reference's GzipDecoder) stops at the first
        # trailer and ignores what follows; a member range here must end at its trailer, so the
        # size is read from the wrong place and the member fails (documented gap)
        ("trailing bytes", good + b"\x00\x01", None),
        ("truncated", good[:len(good) // 2], None),
        ("short", good[:12], 2),
        ("far", far, 9),
    ]


# ---- CPU: the oracle pinned against zlib ----------------------------------------

def test_oracle_matches_zlib(records):
    for name, member, want in corpus(records):
        assert zlib.decompress(member, 31) == want, name
        st, got = oracle_lib.gz_inflate(member)
        assert st == 0 and got == want, name


def test_oracle_reference_fixture(records):
    gz = open(REF_GZ, "rb").read()
    st, got = oracle_lib.gz_inflate(gz)
    assert st == 0 and got == gzip.decompress(gz)
    # cirrussearch layout: an {"index": ...} line before each document; JsonText keeps the 50 texts
    texts = [json.loads(l)["text"] for l in got.decode().splitlines() if "text" in json.loads(l)]
    assert texts == records


def test_oracle_rejects_corrupt_members(records):
    for name, member, want in corrupt_cases(records):
        st, _ = oracle_lib.gz_inflate(member)
        assert st != 0, name
        if want is not None:
            assert st == want, (name, st)
        if name != "trailing bytes":
            with pytest.raises(zlib.error):
                zlib.decompress(member, 31)


def first_member(data):
    """What the reference's GzipDecoder (async-compression 0.3.14, `multiple_members`
    off; gzip_file_provider.rs:18) yields for a file: the first member's bytes, the
    rest of the file ignored.  zlib's decompressobj(31) stops the same way."""
    d = zlib.decompressobj(31)
    out = d.decompress(data) + d.flush()
    assert d.eof
    return out, d.unused_data


def test_member_semantics_vs_reference(native_lib, records):
    """The two deliberate divergences INTEGRATION.md ("Provider: gzip inflate")
    states, pinned against the reference's single-member semantics."""
    from streaming_data_loader_amd import native
    data = payloads(records)["jsonl_x3"]
    # BGZF: the reference stops after the first block; this path inflates every block.
    b = bgzf(data, block=20000)
    ref, rest = first_member(b)
    assert ref == data[:20000] and len(rest) > 0
    off = native.gzip_split_members(b)
    ours = b"".join(oracle_lib.gz_inflate(b[int(off[i]):int(off[i + 1])])[1] for i in range(len(off) - 1))
    assert ours == data == gzip.decompress(b)
    # ...and the reference's output is exactly the first range's
    assert oracle_lib.gz_inflate(b[int(off[0]):int(off[1])]) == (0, ref)
    # `cat a.gz b.gz` as one range: the reference returns a; here the range fails loudly
    a, c = gz_member(data[:7000]), gz_member(data[7000:9000])
    ref, rest = first_member(a + c)
    assert ref == data[:7000] and rest == c
    assert list(native.gzip_split_members(a + c)) == [0, len(a + c)]  # not BGZF: one range
    st, _ = oracle_lib.gz_inflate(a + c)
    assert st != 0
    # one range per file: every file's first (only) member, as the reference reads each file
    assert [oracle_lib.gz_inflate(m)[1] for m in (a, c)] == [first_member(a)[0], first_member(c)[0]]


def test_split_members_host_only(native_lib, records):
    from streaming_data_loader_amd import native
    data = payloads(records)["jsonl_x3"]
    b = bgzf(data, block=20000)
    off = native.gzip_split_members(b)
    assert off[0] == 0 and off[-1] == len(b) and len(off) == (len(data) + 19999) // 20000 + 2
    assert b"".join(zlib.decompress(b[int(off[i]):int(off[i + 1])], 31) for i in range(len(off) - 1)) == data
    plain = gz_member(data)
    assert list(native.gzip_split_members(plain)) == [0, len(plain)]
    assert list(native.gzip_split_members(b"")) == [0]


# ---- GPU: the device inflate against the oracle ------------------------------------

@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a HIP device"
    return t


def device_inflate(torch, db, members, check=True, first=False):
    """members: gzip members (or, with first=True, whole files for sdl_gzip_inflate_first_device)"""
    from streaming_data_loader_amd import native
    buf = b"".join(members)
    off = np.zeros(len(members) + 1, np.uint64)
    np.cumsum([len(m) for m in members], out=off[1:])
    a = np.zeros(len(buf) + 32, np.uint8)
    a[:len(buf)] = np.frombuffer(buf, np.uint8)
    d_gz = torch.from_numpy(a).cuda()
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    call = db.gzip_inflate_first if first else db.gzip_inflate
    rc, out = call(d_gz.data_ptr(), len(buf), d_off.data_ptr(), len(members), check=False)
    if check:
        native.check(rc)
    n = len(members)
    status = np.zeros(n, np.int32)
    mo = np.zeros(n + 1, np.uint32)
    arena = np.zeros(int(out.out_bytes) + 32, np.uint8)
    if n:
        native.d2h(db._h, status, out.d_status, status.nbytes)
        native.d2h(db._h, mo, out.d_member_out, mo.nbytes)
    native.d2h(db._h, arena, out.d_out, arena.nbytes)
    assert (arena[int(out.out_bytes):] == 0).all()
    return rc, out, status, [arena[int(mo[i]):int(mo[i + 1])].tobytes() for i in range(n)], arena


@pytest.mark.gpu
def test_device_inflate_matches_oracle(torch, native_lib, records):
    from streaming_data_loader_amd.device import DeviceBatcher
    db = DeviceBatcher(batch_size=8, sequence_length=128)
    cases = corpus(records)
    rc, out, status, got, arena = device_inflate(torch, db, [m for _, m, _ in cases])
    assert rc == 0 and out.n_bad == 0
    for (name, member, want), st, g in zip(cases, status, got):
        ost, ogot = oracle_lib.gz_inflate(member)
        assert ost == 0 and st == 0, name
        assert g == ogot == want, name
    assert arena[:int(out.out_bytes)].tobytes() == b"".join(w for _, _, w in cases)


@pytest.mark.gpu
def test_first_member_mode_matches_the_reference_decoder(torch, native_lib, records):
    """sdl_gzip_inflate_first_device: one range per FILE, only its first member -- what
    async-compression's GzipDecoder (multiple_members off, gzip_file_provider.rs:18, 64)
    returns, restated by zlib's decompressobj(31) (first_member): `cat a.gz b.gz` -> a,
    a BGZF file -> its first block, a plain file -> all of it, a large single member (the
    chunked path) -> all of it; files of every kind side by side in one call."""
    from streaming_data_loader_amd.device import DeviceBatcher
    db = DeviceBatcher(batch_size=8, sequence_length=128)
    p = payloads(records)
    data = p["jsonl_x3"]
    a, c = gz_member(data[:7000]), gz_member(data[7000:9000])
    files = [
        a + c,                                   # cat a.gz b.gz
        bgzf(data, block=20000),                 # BGZF: the first block
        gz_member(data),                         # one member
        gz_member(p["random"], level=1) + a,     # stored blocks, then another member
        gz_member(b"") + c,                      # an empty first member
        gz_member(p["jsonl"] * 40, level=6),     # >= 1 MiB compressed: the chunked path
        c + a + c,                               # three members
    ]
    assert len(files[5]) >= (1 << 20) // 4
    rc, out, status, got, _ = device_inflate(torch, db, files, first=True)
    assert rc == 0 and (status & 0xFFFF == 0).all(), status
    for i, f in enumerate(files):
        want, _ = first_member(f)
        assert got[i] == want, i
        st, o = oracle_lib.gz_inflate(f[:len(f) - len(first_member(f)[1])])
        assert st == 0 and o == want, i


@pytest.mark.gpu
def test_first_member_mode_false_header_candidates(torch, native_lib, records):
    """A member whose compressed bytes contain the header pattern 1f 8b 08 (stored blocks of
    data that spell it): the first candidate end fails its decode and the next is taken."""
    from streaming_data_loader_amd.device import DeviceBatcher
    db = DeviceBatcher(batch_size=8, sequence_length=128)
    pat = b"\x1f\x8b\x08\x00"
    body = b"x" * 1000 + pat + b"abc" + b"y" * 1000 + pat + b"def" + b"z" * 500  # stored (level 0): in the stream
    first = gz_member(body, level=0)
    assert first.find(b"\x1f\x8b\x08\x00", 10) > 0
    files = [first + gz_member(b"second member"), first]
    rc, out, status, got, _ = device_inflate(torch, db, files, first=True)
    assert rc == 0, status
    assert got == [body, body]


@pytest.mark.gpu
def test_first_member_mode_false_header_in_a_large_member(torch, native_lib, records):
    """A >= 4 MiB member with a planted header pattern whose 4 preceding bytes, read as the
    false range's ISIZE, pass the 1032:1 bound and overflow the 4 GiB arena: the call must
    retry past that candidate, not fail with a capacity error."""
    from streaming_data_loader_amd.device import DeviceBatcher
    db = DeviceBatcher(batch_size=8, sequence_length=128)
    rng = np.random.default_rng(7)
    plant = b"\xf0\xff\xff\xff" + b"\x1f\x8b\x08\x00"  # stored blocks: spelled in the stream (one
    parts = [rng.integers(0, 256, 700_001, dtype=np.uint8).tobytes() for _ in range(8)]  # may straddle a block)
    body = plant.join(parts)
    first = gz_member(body, level=0)
    assert first.find(plant) > 0 and len(first) >= 4 << 20
    files = [first + gz_member(b"second member")]
    rc, out, status, got, _ = device_inflate(torch, db, files, first=True)
    assert rc == 0, status
    assert got == [body]


@pytest.mark.gpu
def test_first_member_mode_trailing_garbage_is_the_stated_limit(torch, native_lib, records):
    from streaming_data_loader_amd.device import DeviceBatcher
    db = DeviceBatcher(batch_size=8, sequence_length=128)
    files = [gz_member(b"hello\n") + b"no header in these trailing bytes"]
    rc, out, status, got, _ = device_inflate(torch, db, files, first=True, check=False)
    assert rc != 0 and int(status[0]) & 0xFFFF != 0


@pytest.mark.gpu
def test_device_reference_fixture_to_records(torch, native_lib, records):
    """data/test.json.gz -> device inflate -> device JsonText: the records the
    reference's provider sends (gzip_file_provider.rs:30-50)."""
    from streaming_data_loader_amd.device import DeviceBatcher
    from streaming_data_loader_amd import native
    db = DeviceBatcher(batch_size=8, sequence_length=128)
    gz = open(REF_GZ, "rb").read()
    rc, out, status, got, _ = device_inflate(torch, db, [gz])
    assert got[0] == gzip.decompress(gz)
    jt = db.json_text(out.d_out, int(out.out_bytes))
    offs = np.zeros(jt.n_records + 1, np.uint64)
    native.d2h(db._h, offs, jt.d_offsets, offs.nbytes)
    text = np.zeros(int(jt.text_bytes), np.uint8)
    native.d2h(db._h, text, jt.d_text, text.nbytes)
    recs = [text[int(offs[i]):int(offs[i + 1])].tobytes().decode() for i in range(jt.n_records)]
    assert recs == records


@pytest.mark.gpu
def test_device_bgzf_and_many_members(torch, native_lib, records):
    from streaming_data_loader_amd.device import DeviceBatcher
    from streaming_data_loader_amd import native
    db = DeviceBatcher(batch_size=8, sequence_length=128)
    data = payloads(records)["jsonl"] * 40  # ~21 MB
    b = bgzf(data)
    off = native.gzip_split_members(b)
    members = [b[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]
    rc, out, status, got, arena = device_inflate(torch, db, members)
    assert rc == 0 and (status == 0).all()
    assert arena[:int(out.out_bytes)].tobytes() == data


@pytest.mark.gpu
def test_device_unaligned_files_as_integration_describes(torch, native_lib, records):
    """INTEGRATION.md's recipe: .json.gz files concatenated with no padding,
    offsets[k] = start of file k, only the base of d_gz aligned.  Every file
    length here is odd, so no member after the first starts 16-B aligned."""
    from streaming_data_loader_amd.device import DeviceBatcher
    db = DeviceBatcher(batch_size=8, sequence_length=128)
    lines = payloads(records)["jsonl"]
    files, want = [], []
    for k in range(7):
        d = lines[k * 1111:(k + 1) * 1111 + 37 * k] + b"\n"
        m = gz_member(d, level=(1, 6, 9)[k % 3], name=b"f%d.json" % k if k % 2 else b"")
        if len(m) % 2 == 0:
            m = gz_member(d, level=(1, 6, 9)[k % 3], name=b"f%d.jsonx" % k)
        assert len(m) % 2 == 1
        files.append(m)
        want.append(d)
    rc, out, status, got, arena = device_inflate(torch, db, files)
    assert rc == 0 and (status == 0).all()
    assert got == want and [first_member(f)[0] for f in files] == want


@pytest.mark.gpu
def test_device_rejects_corrupt_members(torch, native_lib, records):
    from streaming_data_loader_amd.device import DeviceBatcher
    from streaming_data_loader_amd import native
    db = DeviceBatcher(batch_size=8, sequence_length=128)
    good = gz_member(payloads(records)["jsonl"][:5000])
    cases = corrupt_cases(records)
    members = [good] + [m for _, m, _ in cases] + [good]
    rc, out, status, got, _ = device_inflate(torch, db, members, check=False)
    assert rc == native.SDL_ERR_DATA and out.n_bad == len(cases)
    assert status[0] == 0 and status[-1] == 0 and got[0] == got[-1] == zlib.decompress(good, 31)
    for (name, member, want), st in zip(cases, status[1:-1]):
        ost, _ = oracle_lib.gz_inflate(member)
        assert st != 0, name
        if want is not None:
            assert st == want == ost, (name, st, ost)
    # the handle stays usable after a failed call
    rc, out, status, got, _ = device_inflate(torch, db, [good])
    assert rc == 0 and got[0] == zlib.decompress(good, 31)


# ---- GPU: large single members, inflated in chunks (the reference's input shape) ----

def big_lines(records, mib, seed=0):
    rng = random.Random(seed)
    out, size = [], 0
    while size < mib << 20:
        t = records[rng.randrange(len(records))]
        ln = json.dumps({"id": len(out), "text": t}).encode() + b"\n"
        out.append(ln)
        size += len(ln)
    return b"".join(out)


def chunked_cases(records):
    """(name, member, expected bytes): members of >= 1 MiB compressed take the
    chunked path (GZ_SPLIT_MIN in sdl_batcher.cpp)."""
    rng = random.Random(3)
    lines = big_lines(records, 8)
    noise = bytes(rng.randrange(256) for _ in range(1_200_000))
    cases = [
        ("jsonl l6", gz_member(lines, 6), lines),
        ("jsonl l1", gz_member(lines, 1), lines),
        ("jsonl l9 filtered", gz_member(lines, 9, zlib.Z_FILTERED), lines),
        ("jsonl huffman-only", gz_member(lines[:3_000_000], 6, zlib.Z_HUFFMAN_ONLY), lines[:3_000_000]),
        ("jsonl rle", gz_member(lines[:4_000_000], 6, zlib.Z_RLE), lines[:4_000_000]),
        ("jsonl header fields + full flushes", gz_member(lines, 6, name=b"dump.json", comment=b"x", flags=2,
                                                         flush_every=1 << 20), lines),
        # no dynamic blocks to find: every chunk is decoded again from its predecessor's end
        ("fixed codes", gz_member(lines[:3_000_000], 6, zlib.Z_FIXED), lines[:3_000_000]),
        ("stored + text", gz_member(noise + lines[:2_000_000], 6), noise + lines[:2_000_000]),
        # a block that outgrows a chunk's slot (long runs): the one-wave path takes the member
        ("runs", gz_member(noise + b"a" * 5_000_000 + lines[:500_000], 9), noise + b"a" * 5_000_000 + lines[:500_000]),
    ]
    for name, m, _ in cases:
        assert len(m) >= 1 << 20, (name, len(m))
    return cases


@pytest.mark.gpu
def test_device_chunked_members_match_zlib(torch, native_lib, records):
    from streaming_data_loader_amd.device import DeviceBatcher
    db = DeviceBatcher(batch_size=8, sequence_length=128)
    for name, member, want in chunked_cases(records):
        rc, out, status, got, _ = device_inflate(torch, db, [member])
        assert rc == 0 and status[0] == 0, (name, rc, status[0])
        assert got[0] == want == zlib.decompress(member, 31), name


@pytest.mark.gpu
def test_device_chunked_member_among_small_ones(torch, native_lib, records):
    """One call: small members (one wave each) around a large one (chunked),
    the reference fixture among them."""
    from streaming_data_loader_amd.device import DeviceBatcher
    db = DeviceBatcher(batch_size=8, sequence_length=128)
    lines = big_lines(records, 6, seed=1)
    ref = open(REF_GZ, "rb").read()
    small = [gz_member(lines[:5000]), ref, gz_member(b"")]
    members = [small[0], gz_member(lines), small[1], gz_member(lines[::-1]), small[2]]
    want = [zlib.decompress(m, 31) for m in members]
    rc, out, status, got, arena = device_inflate(torch, db, members)
    assert rc == 0 and (status == 0).all()
    assert got == want


@pytest.mark.gpu
def test_device_chunked_member_errors(torch, native_lib, records):
    """Damage in a large member fails it (not its neighbours) with the oracle's
    status where the reason does not depend on where a decoder notices it."""
    from streaming_data_loader_amd.device import DeviceBatcher
    from streaming_data_loader_amd import native
    db = DeviceBatcher(batch_size=8, sequence_length=128)
    lines = big_lines(records, 6, seed=2)
    good = gz_member(lines)
    bad_crc = bytearray(good)
    bad_crc[-8] ^= 1
    bad_size = bytearray(good)
    bad_size[-2] ^= 1                      # ISIZE still within DEFLATE's bound
    trunc = good[:len(good) * 2 // 3]
    trailing = good + b"\x00\x01"
    mid = bytearray(good)
    mid[len(good) // 2] ^= 0xFF            # damage deep inside: some GZ_E_* (where it is noticed varies)
    cases = [("crc", bytes(bad_crc), 13), ("isize", bytes(bad_size), None), ("truncated", trunc, None),
             ("trailing", trailing, None), ("middle", bytes(mid), None)]
    small = gz_member(lines[:3000])
    for name, m, want in cases:
        rc, out, status, got, _ = device_inflate(torch, db, [small, m, small], check=False)
        ost, _ = oracle_lib.gz_inflate(m)
        assert rc == native.SDL_ERR_DATA and out.n_bad == 1, name
        assert status[0] == 0 and status[2] == 0 and got[0] == got[2] == lines[:3000], name
        assert status[1] != 0 and ost != 0, name
        if want is not None:
            assert status[1] == want == ost, (name, status[1], ost)
    rc, out, status, got, _ = device_inflate(torch, db, [good])  # the handle stays usable
    assert rc == 0 and got[0] == lines


def decoy_member(records):
    """A >= 1 MiB member whose middle is a stored block full of complete final dynamic-Huffman
    DEFLATE streams (the 'decoys'): a chunk whose header search lands in the stored bytes picks
    a decoy and decodes a final block that is not the member's.  Raw DEFLATE is assembled by
    hand: text (full flush, byte-aligned) + stored block of decoys + text (final)."""
    lines = big_lines(records, 4, seed=5)
    head, tail = lines[:3_000_000], lines[3_000_000:]
    rng = random.Random(11)
    decoys = []
    while sum(map(len, decoys)) < 60_000:
        text = bytes(rng.choice(b"abcdefghij klmnop,.\n") for _ in range(rng.randrange(600, 1400)))
        d = zlib.compressobj(9, zlib.DEFLATED, -15)
        raw = d.compress(text) + d.flush()
        assert raw[0] & 7 == 0b101  # BFINAL 1, BTYPE 10 (dynamic)
        decoys.append(raw)
    payload = b"".join(decoys)[:65535]
    a = zlib.compressobj(6, zlib.DEFLATED, -15)
    deflate = a.compress(head) + a.flush(zlib.Z_FULL_FLUSH)  # ends byte-aligned, not final
    n = len(payload)
    deflate += bytes([0]) + n.to_bytes(2, "little") + (n ^ 0xFFFF).to_bytes(2, "little") + payload
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    deflate += c.compress(tail) + c.flush()
    data = head + payload + tail
    member = (b"\x1f\x8b\x08\x00\x00\x00\x00\x00\x00\x03" + deflate
              + (zlib.crc32(data) & 0xFFFFFFFF).to_bytes(4, "little") + (len(data) & 0xFFFFFFFF).to_bytes(4, "little"))
    assert len(member) >= 1 << 20 and zlib.decompress(member, 31) == data
    return member, data


def test_decoy_member_is_valid_gzip(records):
    member, data = decoy_member(records)
    assert oracle_lib.gz_inflate(member) == (0, data)


@pytest.mark.gpu
def test_device_chunked_member_with_decoy_final_blocks(torch, native_lib, records):
    """chunks that start from a wrong header pick may decode a final block; the
    trailer CRC must not come from whichever chunk wrote last.  Repeated to catch a race."""
    from streaming_data_loader_amd.device import DeviceBatcher
    db = DeviceBatcher(batch_size=8, sequence_length=128)
    member, data = decoy_member(records)
    for _ in range(6):
        rc, out, status, got, _ = device_inflate(torch, db, [member])
        assert rc == 0 and status[0] == 0, (rc, status[0])
        assert got[0] == data
