"""Pure-Python restatement of the reference's RNG pieces, for goldens and
tests (independent of the C oracle):

  rand_chacha 0.3.1  ChaCha12Rng / StdRng::from_seed (64-bit block counter,
                     stream 0, words in block order; BlockRng next_u64 = two
                     words, low first);
  rand_pcg 0.3       Pcg32::new(state, stream) (rand's and rand_distr's test rng);
  rand_distr 0.4.3   StandardNormal for f64: utils::ziggurat with the
                     ZIG_NORM_X / ZIG_NORM_F tables of rand's
                     ziggurat_tables.py (printed with %.18f), rand 0.8.5
                     Open01 / Standard f64 for the tail and wedge draws.

Pinned by rand_distr's value-stability vector for StandardNormal (seed 213):
tests/test_rand_mode.py.
"""
import math
import struct

M32, M64 = 0xFFFFFFFF, (1 << 64) - 1


def _rotl(x, r):
    return ((x << r) | (x >> (32 - r))) & M32


def chacha_block(key, counter, stream=0, rounds=12):
    s = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + list(key) + \
        [counter & M32, counter >> 32, stream & M32, stream >> 32]
    x = list(s)

    def qr(a, b, c, d):
        x[a] = (x[a] + x[b]) & M32; x[d] = _rotl(x[d] ^ x[a], 16)
        x[c] = (x[c] + x[d]) & M32; x[b] = _rotl(x[b] ^ x[c], 12)
        x[a] = (x[a] + x[b]) & M32; x[d] = _rotl(x[d] ^ x[a], 8)
        x[c] = (x[c] + x[d]) & M32; x[b] = _rotl(x[b] ^ x[c], 7)
    for _ in range(rounds // 2):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return [(a + b) & M32 for a, b in zip(x, s)]


class StdRng:
    def __init__(self, seed32):
        self.key = [int.from_bytes(seed32[4 * i:4 * i + 4], "little") for i in range(8)]
        self.ctr, self.buf = 0, []

    def u32(self):
        if not self.buf:
            self.buf = chacha_block(self.key, self.ctr)
            self.ctr += 1
        return self.buf.pop(0)

    def u64(self):
        lo = self.u32()
        return lo | self.u32() << 32


def row_seed(seed, record, chunk):
    return seed.to_bytes(8, "little") + record.to_bytes(8, "little") + chunk.to_bytes(4, "little") + bytes(12)


class Pcg32:
    def __init__(self, state, stream):
        self.inc = ((stream << 1) | 1) & M64
        self.state = (state + self.inc) & M64
        self.state = (self.state * 6364136223846793005 + self.inc) & M64

    def u32(self):
        s = self.state
        self.state = (s * 6364136223846793005 + self.inc) & M64
        rot, xsh = s >> 59, (((s >> 18) ^ s) >> 27) & M32
        return ((xsh >> rot) | (xsh << ((32 - rot) & 31))) & M32

    def u64(self):
        lo = self.u32()
        return lo | self.u32() << 32


ZIG_R, ZIG_V = 3.6541528853610088, 0.00492867323399


def _tables():
    f = lambda x: math.exp(-x * x / 2.0)  # noqa: E731
    x = [0.0] * 257
    x[0], x[1] = ZIG_V / f(ZIG_R), ZIG_R
    for i in range(2, 256):
        x[i] = math.sqrt(-2.0 * math.log(ZIG_V / x[i - 1] + f(x[i - 1])))
    return [float("%.18f" % v) for v in x], [float("%.18f" % f(v)) for v in x]


ZX, ZF = _tables()


def _f64(bits):
    return struct.unpack("<d", struct.pack("<Q", bits))[0]


def std_normal(rng, stats=None):
    """One StandardNormal f64; stats (dict) counts the fast / wedge / tail exits."""
    while True:
        bits = rng.u64()
        i = bits & 0xFF
        u = _f64((bits >> 12) | (1024 << 52)) - 3.0
        x = u * ZX[i]
        if abs(x) < ZX[i + 1]:
            if stats is not None:
                stats["fast"] = stats.get("fast", 0) + 1
            return x
        if i == 0:
            xt, yt = 1.0, 0.0
            while -2.0 * yt < xt * xt:
                a = _f64((rng.u64() >> 12) | (1023 << 52)) - (1.0 - 2.0 ** -53)
                c = _f64((rng.u64() >> 12) | (1023 << 52)) - (1.0 - 2.0 ** -53)
                xt, yt = math.log(a) / ZIG_R, math.log(c)
            if stats is not None:
                stats["tail"] = stats.get("tail", 0) + 1
            return xt - ZIG_R if u < 0.0 else ZIG_R - xt
        g = (rng.u64() >> 11) * (1.0 / (1 << 53))
        if ZF[i + 1] + (ZF[i] - ZF[i + 1]) * g < math.exp(-x * x / 2.0):
            if stats is not None:
                stats["wedge"] = stats.get("wedge", 0) + 1
            return x
        if stats is not None:
            stats["retry"] = stats.get("retry", 0) + 1


def sat_usize(d):
    """Rust `f64 as usize`: truncation toward zero, NaN and negatives -> 0."""
    if not d > 0.0:
        return 0
    return min(int(d), M64)
