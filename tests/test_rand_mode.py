"""The optional rand-compatible MLM mode (rng_mode = 1): BertData::mask_batch's
`position_base.shuffle(&mut thread_rng())` (rust/src/models/bert_data.rs:40-43)
with thread_rng replaced by `StdRng::from_seed(row_seed)` per row, row_seed =
seed | record | chunk (little-endian u64, u64, u32, 12 zero bytes).

rand 0.8.5 / rand_chacha 0.3.1 are not vendored and cargo is absent, so the
restatement (oracle/orc_batcher.c) is pinned by the published vectors of the
pieces it is built from:
  - ChaCha20 block function: RFC 7539 §2.3.2 and appendix A.1 test vector #1;
  - StdRng (ChaCha12, 64-bit counter, output order): rand's
    test_stdrng_construction (from_seed -> next_u64, from_rng -> next_u64);
  - gen_index / gen_range(0..n) / shuffle: rand's value_stability_slice
    (Pcg32 test rng seeded 414, 13 elements), through the pure-Python
    restatement below, which then checks the C oracle's positions.
The span mode (rng_mode = 1 with task span): T5Data::put_data's
random_data_gap / random_data_size (rust/src/models/t5_data.rs:165-176) draw
rand_distr 0.4.3 StandardNormal f64 samples from the same per-row StdRng, gap
then size per pass.  The ziggurat restatement (oracle/orc_batcher.c
std_normal, tests/golden/randref.py) is pinned by rand_distr's value-stability
vector (tests/value_stability.rs normal_distributions_stability, seed 213 of
its Pcg32 test rng); the tail and wedge exits are exercised beyond it by the
two restatements agreeing on long streams.
The device path is checked against the oracle in test_gpu_rand_mode.py.
"""
import ctypes
import json
import os

import numpy as np

import oracle_lib

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
M64 = (1 << 64) - 1


def chacha(key_words, counter, stream, rounds):
    out = (ctypes.c_uint32 * 16)()
    oracle_lib.lib().orc_chacha_block((ctypes.c_uint32 * 8)(*key_words), counter, stream, rounds, out)
    return list(out)


def words(b):
    return [int.from_bytes(b[4 * i:4 * i + 4], "little") for i in range(len(b) // 4)]


def test_chacha20_rfc7539_block():
    key = words(bytes(range(32)))
    nonce = words(bytes.fromhex("000000090000004a00000000"))
    got = chacha(key, 1 | nonce[0] << 32, nonce[1] | nonce[2] << 32, 20)
    assert got == [0xe4e7f110, 0x15593bd1, 0x1fdd0f50, 0xc47120a3, 0xc7f4d1c7, 0x0368c033, 0x9aaa2204, 0x4e6cd4c3,
                   0x466482d2, 0x09aa9f07, 0x05d7c214, 0xa2028bd9, 0xd19c12b5, 0xb94e16de, 0xe883d0cb, 0x4e3c50a2]
    # A.1 #1: all-zero key and nonce, counter 0 (keystream 76 b8 e0 ad a0 f1 3d 90 ...)
    assert chacha([0] * 8, 0, 0, 20)[:4] == [0xade0b876, 0x903df1a0, 0xe56a5d40, 0x28bd8653]


class StdRng:
    """rand_chacha's ChaCha12Rng over the oracle's block function."""

    def __init__(self, seed32):
        self.key, self.ctr, self.buf = words(seed32), 0, []

    def u32(self):
        if not self.buf:
            self.buf = chacha(self.key, self.ctr, 0, 12)
            self.ctr += 1
        return self.buf.pop(0)

    def u64(self):
        lo = self.u32()
        return lo | self.u32() << 32


def test_stdrng_construction_vectors():
    seed = bytes([1, 0, 0, 0, 23, 0, 0, 0, 200, 1, 0, 0, 210, 30, 0, 0] + [0] * 16)
    r0 = StdRng(seed)
    assert r0.u64() == 10719222850664546238
    assert oracle_lib.lib().orc_stdrng_first_u64((ctypes.c_uint8 * 32)(*seed)) == 10719222850664546238
    # StdRng::from_rng(rng0): fill_bytes takes the next 8 words, little-endian
    seed1 = b"".join(r0.u32().to_bytes(4, "little") for _ in range(8))
    assert StdRng(seed1).u64() == 14064965282130556830


class Pcg32:
    """rand_pcg::Pcg32::new(state, stream) (rand's crate::test::rng)."""

    def __init__(self, state, stream):
        self.inc = ((stream << 1) | 1) & M64
        self.state = (state + self.inc) & M64
        self._step()

    def _step(self):
        self.state = (self.state * 6364136223846793005 + self.inc) & M64

    def u32(self):
        s = self.state
        self._step()
        rot, xsh = s >> 59, (((s >> 18) ^ s) >> 27) & 0xFFFFFFFF
        return ((xsh >> rot) | (xsh << ((32 - rot) & 31))) & 0xFFFFFFFF


def gen_index(rng, n):
    zone = ((n << (32 - n.bit_length())) & 0xFFFFFFFF) - 1
    while True:
        m = rng.u32() * n
        if m & 0xFFFFFFFF <= zone:
            return m >> 32


def shuffle(a, rng):
    for i in range(len(a) - 1, 0, -1):
        j = gen_index(rng, i + 1)
        a[i], a[j] = a[j], a[i]


def test_shuffle_value_stability():
    nums = list(range(13))
    shuffle(nums, Pcg32(414, 11634580027462260723))
    assert nums == [9, 5, 3, 10, 7, 12, 8, 11, 6, 4, 0, 2, 1]


def row_seed(seed, record, chunk):
    return seed.to_bytes(8, "little") + record.to_bytes(8, "little") + chunk.to_bytes(4, "little") + bytes(12)


def test_oracle_positions_match_restatement():
    L = oracle_lib.lib()
    for seed, rec, chunk, S in ((0, 0, 0, 128), (1234, 7, 3, 512), (2 ** 63 + 5, 10 ** 7 + 11, 0, 1024), (9, 1, 1, 2)):
        want = list(range(S))
        shuffle(want, StdRng(row_seed(seed, rec, chunk)))
        got = (ctypes.c_uint32 * S)()
        L.orc_rand_positions(seed, rec, chunk, S, got)
        assert list(got) == want, (seed, rec, chunk, S)


def test_oracle_batcher_rand_mode(oracle_tok, records):
    """GenTokenizer + BertData in rand mode at the reference CPU config (S=128,
    B=8): the oracle's masks are the first mask_length shuffled positions of
    the restated StdRng, non-pad ids only."""
    enc = oracle_lib.Encoder("bert", oracle_tok)
    plain = oracle_lib.OracleBatcherEx(enc, oracle_lib.MLM, 8, 128, mask_length=0, seed=77, rng_mode=1)
    rand = oracle_lib.OracleBatcherEx(enc, oracle_lib.MLM, 8, 128, seed=77, rng_mode=1)
    philox = oracle_lib.OracleBatcherEx(enc, oracle_lib.MLM, 8, 128, seed=77, rng_mode=0)
    n_rows = n_masked = 0
    for rec, t in enumerate(records + [None]):
        a = plain.push(t) if t is not None else plain.flush()
        b = rand.push(t) if t is not None else rand.flush()
        c = philox.push(t) if t is not None else philox.flush()
        assert (a is None) == (b is None) == (c is None)
        if a is None:
            continue
        for r in range(8):
            ids = a["input_ids"][r]
            if not ids.any():
                continue
            n_rows += 1
        assert not np.array_equal(b["labels"], c["labels"]) or not b["labels"].any()
        n_masked += int((b["labels"] != -100).sum())
    assert n_rows > 20 and n_masked > 100


def test_oracle_rand_rows_exact(oracle_tok, records):
    """Row by row: the record index and chunk of every emitted row are known
    (first_record 0, records in order), so the expected masked row is rebuilt
    from the unmasked one and the restated shuffle."""
    enc = oracle_lib.Encoder("bert", oracle_tok)
    S, B, k = 128, 4, int(np.float32(128) * np.float32(0.15))
    plain = oracle_lib.OracleBatcherEx(enc, oracle_lib.MLM, B, S, mask_length=0, seed=5, rng_mode=1)
    rand = oracle_lib.OracleBatcherEx(enc, oracle_lib.MLM, B, S, seed=5, rng_mode=1)
    # (record, chunk) of each row in emission order: records with >= 64 framed ids, chunked by S
    tags = []
    for rec, t in enumerate(records):
        n = len(oracle_tok.encode(t)) + 3  # [CLS] + encode (with its own [CLS] [SEP]) + [SEP] [SEP]
        if n >= 64:
            tags += [(rec, c) for c in range((n + S - 1) // S)]
    rows_plain, rows_rand = [], []
    for t in records + [None]:
        a = plain.push(t) if t is not None else plain.flush()
        b = rand.push(t) if t is not None else rand.flush()
        if a is not None:
            rows_plain += [a["input_ids"][i].copy() for i in range(B)]
            rows_rand += [(b["input_ids"][i].copy(), b["labels"][i].copy()) for i in range(B)]
    checked = 0
    for (rec, chunk), ids, (mids, labs) in zip(tags, rows_plain, rows_rand):
        pos = list(range(S))
        shuffle(pos, StdRng(row_seed(5, rec, chunk)))
        want_ids, want_lab = ids.copy(), np.full(S, -100, np.int32)
        for p in pos[:k]:
            if ids[p] != 0:
                want_lab[p] = ids[p]
                want_ids[p] = 103
        np.testing.assert_array_equal(mids, want_ids)
        np.testing.assert_array_equal(labs, want_lab)
        checked += 1
    assert checked >= 20


# ---- span: rand_distr StandardNormal over the row's StdRng ------------------------
import randref  # noqa: E402  (tests/golden on sys.path via conftest)

RAND_DISTR_NORMAL_213 = [-0.11844188827977231, 0.7813779637772346, 0.06563993969580051, -1.1932899004186373]


def test_standard_normal_value_stability():
    """rand_distr 0.4.3 tests/value_stability.rs: StandardNormal f64 from
    Pcg32::new(213, 11634580027462260723) -- bit for bit, both restatements."""
    r = randref.Pcg32(213, 11634580027462260723)
    assert [randref.std_normal(r) for _ in range(4)] == RAND_DISTR_NORMAL_213
    out = np.zeros(4)
    oracle_lib.lib().orc_normal_pcg32(213, 11634580027462260723, 4, out.ctypes.data)
    assert out.tolist() == RAND_DISTR_NORMAL_213
    # Normal::new(2.0, 0.5) of the same draws (mean + std * z), as the vector file lists
    assert [2.0 + 0.5 * z for z in RAND_DISTR_NORMAL_213][0] == 1.940779055860114


def test_ziggurat_tables_published_head():
    """The first entries of rand_distr's ziggurat_tables.rs as printed there (%.18f)."""
    assert randref.ZX[:4] == [3.910757959537090045, 3.654152885361008796, 3.449278298560964462, 3.320244733839166074]
    assert randref.ZF[:3] == [0.000477467764586655, 0.001260285930498598, 0.002609072746106363]
    assert randref.ZX[256] == 0.0 and randref.ZF[256] == 1.0


def test_oracle_row_normals_match_restatement():
    """Long per-row streams (every exit of the ziggurat taken) agree bit for bit."""
    stats = {}
    for seed, rec, chunk in ((1234, 0, 0), (1234, 17, 3), (2 ** 63 + 5, 10 ** 7 + 11, 1)):
        n = 30000
        r = randref.StdRng(randref.row_seed(seed, rec, chunk))
        want = [randref.std_normal(r, stats) for _ in range(n)]
        got = np.zeros(n)
        oracle_lib.lib().orc_normal_row(seed, rec, chunk, n, got.ctypes.data)
        assert got.tolist() == want, (seed, rec, chunk)
    assert stats["tail"] > 0 and stats["wedge"] > 50 and stats["retry"] > 50, stats
    z = np.array(want)
    assert abs(z.mean()) < 0.03 and abs(z.std() - 1.0) < 0.03


def test_oracle_span_rand_batches_match_golden(records):
    """GenTokenizer + T5Data in rng_mode 1 at S=128 B=8 over the fixture stream
    vs tests/golden/span_rand_s128_b8.npz (ids from tokenizers, draws from randref)."""
    g = np.load(os.path.join(GOLDEN, "span_rand_s128_b8.npz"))
    tok = oracle_lib.T5Tok()
    ob = oracle_lib.OracleBatcherEx(oracle_lib.Encoder("t5", tok), oracle_lib.SPAN, 8, 128, seed=1234, rng_mode=1)
    got = [r for r in (ob.push(t) for t in records) if r is not None]
    got.append(ob.flush())
    assert len(got) == int(g["n_batches"])
    for i, r in enumerate(got):
        assert r["rows"] == int(g[f"b{i}_rows"])
        for k in ("input_ids", "attention_mask", "labels"):
            np.testing.assert_array_equal(r[k], g[f"b{i}_{k}"], err_msg=f"batch {i} {k}")
    assert ob.span_errors() == int(g["span_errors"])
    philox = np.load(os.path.join(GOLDEN, "span_s128_b8.npz"))
    assert not np.array_equal(philox["b0_labels"], g["b0_labels"])
