// tok_device.hpp -- device helpers shared by the tokenize kernels
// (tokenize_wordpiece.hip, tokenize_bpe.hip): the LDS text window of a chunk,
// 16-byte register words, the cuckoo vocab probe and UTF-8 decoding.
#pragma once

#include "common.hpp"
#include "device_util.hpp"

namespace sdl {
namespace {

typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint64_t lds_u64;

constexpr int RBITS_WORDS = WIN / 32;  // 34

struct Ctx {
    const DevTok *T;
    const lds_u8 *win;      // LDS window [w0, w0 + WIN)
    const lds_u32 *rbits;   // LDS bitmap: record starts in the window
    int64_t w0;
    const uint8_t *text;
    int64_t N;
    const uint64_t *off;
    int64_t R;

    __device__ __forceinline__ bool in_win(int64_t p) const { return (uint64_t)(p - w0) < (uint64_t)WIN; }
    __device__ __forceinline__ uint32_t byte(int64_t p) const {
        uint32_t r;
        if (in_win(p)) r = win[p - w0];
        else r = __builtin_nontemporal_load(text + p);
        return r;
    }
    // true when a record starts at p (0 <= p <= N)
    __device__ __forceinline__ bool rstart(int64_t p) const {
        if (in_win(p)) {
            const int i = (int)(p - w0);
            return (rbits[i >> 5] >> (i & 31)) & 1u;
        }
        int64_t lo = 0, hi = R;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if ((int64_t)off[mid] < p) lo = mid + 1; else hi = mid;
        }
        return (int64_t)off[lo] == p;
    }
};

__device__ __forceinline__ uint32_t hinit(uint32_t len, uint32_t cont) { return ph_init(len, cont); }
__device__ __forceinline__ uint32_t hmix(uint32_t h, uint32_t w) { return ph_mix(h, w); }
__device__ __forceinline__ uint32_t hfinal(uint32_t h) { return ph_final(h); }

// ---- 16-byte register words ---------------------------------------------------
struct W16 {
    uint32_t x, y, z, w;
};

// bytes [k, k + 16) of a (zero beyond 16), k in [0, 16)
__device__ __forceinline__ W16 shift_right_bytes(const W16 &a, int k) {
    const int q = k >> 2;
    const uint32_t r = (uint32_t)(k & 3);
    auto word = [&](int j) -> uint32_t { return j == 0 ? a.x : j == 1 ? a.y : j == 2 ? a.z : j == 3 ? a.w : 0u; };
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = __builtin_amdgcn_alignbyte(word(i + q + 1), word(i + q), r);
    return W16{o[0], o[1], o[2], o[3]};
}

// keep the first n bytes (n in [0, 16])
__device__ __forceinline__ W16 keep_bytes(const W16 &a, int n) {
    auto m = [&](int i) -> uint32_t {
        const int k = n - 4 * i;
        return k >= 4 ? 0xFFFFFFFFu : k <= 0 ? 0u : (0xFFFFFFFFu >> (32 - 8 * k));
    };
    return W16{a.x & m(0), a.y & m(1), a.z & m(2), a.w & m(3)};
}

// SWAR: 0x80 in every byte of x that is an ASCII letter or digit
__device__ __forceinline__ uint32_t swar_alnum(uint32_t x) {
    const uint32_t hi = x & 0x80808080u;
    const uint32_t l = (x | 0x20202020u) & 0x7F7F7F7Fu;
    const uint32_t ge_a = (l + 0x1F1F1F1Fu) & 0x80808080u;   // l >= 0x61
    const uint32_t le_z = ~(l + 0x05050505u) & 0x80808080u;  // l <= 0x7A
    const uint32_t d = x & 0x7F7F7F7Fu;
    const uint32_t ge_0 = (d + 0x50505050u) & 0x80808080u;   // d >= 0x30
    const uint32_t le_9 = ~(d + 0x46464646u) & 0x80808080u;  // d <= 0x39
    return ((ge_a & le_z) | (ge_0 & le_9)) & ~hi;
}
// SWAR lower-case of ASCII A-Z
__device__ __forceinline__ uint32_t swar_lower(uint32_t x) {
    const uint32_t d = x & 0x7F7F7F7Fu;
    const uint32_t ge_A = (d + 0x3F3F3F3Fu) & 0x80808080u;   // d >= 0x41
    const uint32_t le_Z = ~(d + 0x25252525u) & 0x80808080u;  // d <= 0x5A
    const uint32_t up = ge_A & le_Z & ~(x & 0x80808080u);
    return x | (up >> 2);
}
// 4-bit mask from the 0x80 bits of a SWAR result
__device__ __forceinline__ uint32_t msb4(uint32_t m) {
    return ((m >> 7) & 1u) | ((m >> 14) & 2u) | ((m >> 21) & 4u) | ((m >> 28) & 8u);
}

// ---- byte-parallel helpers: 4 bytes per dword, predicates in bit 7 of each byte
constexpr uint32_t B7 = 0x80808080u;
__device__ __forceinline__ uint32_t nzb(uint32_t x) { return (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & B7; }
__device__ __forceinline__ uint32_t bit7(uint32_t x, int k) { return (x << (7 - k)) & B7; }
__device__ __forceinline__ uint32_t fullb(uint32_t m) { return (m >> 7) * 0xFFu; }
__device__ __forceinline__ uint32_t expand4(uint32_t b4) { return ((b4 * 0x00204081u) & 0x01010101u) << 7; }
__device__ __forceinline__ uint32_t gather4(uint32_t m) { return ((((m >> 7) & 0x01010101u) * 0x00204081u) >> 21) & 0xFu; }
__device__ __forceinline__ uint32_t gather16(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return gather4(a) | gather4(b) << 4 | gather4(c) << 8 | gather4(d) << 12;
}
// bytes y < 0x80: y >= lo, lo <= y <= hi
__device__ __forceinline__ uint32_t ge7(uint32_t y, uint32_t lo) { return (y + (0x80u - lo) * 0x01010101u) & B7; }
__device__ __forceinline__ uint32_t in7(uint32_t y, uint32_t lo, uint32_t hi) { return ge7(y, lo) & ~ge7(y, hi + 1); }
// 4 bytes of values < 16 -> 4 nibbles (byte k -> bits 4k..4k+3)
__device__ __forceinline__ uint32_t nibpack4(uint32_t x) {
    const uint32_t z = x | (x >> 4);
    return (z & 0xFFu) | ((z >> 8) & 0xFF00u);
}
// 16-bit mask -> bit 4i per bit i
__device__ __forceinline__ uint64_t nib_spread(uint32_t m16) {
    uint64_t x = m16;
    x = (x | (x << 24)) & 0x000000FF000000FFull;
    x = (x | (x << 12)) & 0x000F000F000F000Full;
    x = (x | (x << 6)) & 0x0303030303030303ull;
    return (x | (x << 3)) & 0x1111111111111111ull;
}

// Strict UTF-8 decode of the char at lead byte b = byte(p); must not cross a
// record start.  Invalid -> U+FFFD (class DEL), 1 byte.
__device__ __forceinline__ uint32_t decode(const Ctx &C, int64_t p, uint32_t b, int *len) {
    int n;
    uint32_t c;
    if ((b & 0xE0u) == 0xC0u) { n = 2; c = b & 0x1Fu; }
    else if ((b & 0xF0u) == 0xE0u) { n = 3; c = b & 0x0Fu; }
    else if ((b & 0xF8u) == 0xF0u) { n = 4; c = b & 0x07u; }
    else { *len = 1; return 0xFFFDu; }
    if (p + n > C.N) { *len = 1; return 0xFFFDu; }
    for (int k = 1; k < n; ++k) {
        const uint32_t x = C.byte(p + k);
        if ((x & 0xC0u) != 0x80u || C.rstart(p + k)) { *len = 1; return 0xFFFDu; }
        c = (c << 6) | (x & 0x3Fu);
    }
    *len = n;
    return c;
}

// Longest added token starting at p that does not cross a record start; -1 if
// none.  Added tokens never overlap: their first byte occurs nowhere else in
// them (checked on the host), so leftmost-longest matching is local.
__device__ __forceinline__ int special_match(const Ctx &C, int64_t p) {
    const DevTok &T = *C.T;
    int best = -1, best_len = 0;
    for (int k = 0; k < T.n_special; ++k) {
        const int l = T.special_len[k];
        if (p + l > C.N || l <= best_len) continue;
        bool ok = true;
        for (int j = 1; j < l && ok; ++j) ok = C.byte(p + j) == T.special_bytes[k][j] && !C.rstart(p + j);
        if (ok) { best = k; best_len = l; }
    }
    return best;
}

// Reads both cuckoo slots of hash h (4 independent 16-B loads).
struct Probe {
    uint4 a1, b1, a2, b2;
};
__device__ __forceinline__ Probe probe_load(const DevTok &T, uint32_t h) {
    const uint4 *e1 = reinterpret_cast<const uint4 *>(T.slots + cuckoo_slot1(h, T.slot_mask));
    const uint4 *e2 = reinterpret_cast<const uint4 *>(T.slots + cuckoo_slot2(h, T.slot_mask));
    return Probe{e1[0], e1[1], e2[0], e2[1]};
}
// (one OR of differences and one compare: a chain of && costs a scalar mask op per term)
__device__ __forceinline__ uint32_t slot_diff(const uint4 &a, const uint4 &b, uint32_t key, const W16 &c) {
    return (a.x ^ key) | (b.x ^ c.x) | (b.y ^ c.y) | (b.z ^ c.z) | (b.w ^ c.w) | (a.y >> 31);
}
__device__ __forceinline__ bool slot_match(const uint4 &a, const uint4 &b, uint32_t key, const W16 &c) {
    return slot_diff(a, b, key, c) == 0u;
}
// id of the piece (payload <= 16 bytes in c, zero padded) or -1: exact
__device__ __forceinline__ int probe_result(const Probe &P, uint32_t key, const W16 &c) {
    const uint32_t d1 = slot_diff(P.a1, P.b1, key, c), d2 = slot_diff(P.a2, P.b2, key, c);
    const int r2 = d2 == 0u ? (int32_t)P.a2.y : -1;
    return d1 == 0u ? (int32_t)P.a1.y : r2;
}
__device__ __forceinline__ uint32_t hash16(const W16 &c, uint32_t n, uint32_t cont) {
    uint32_t h = hinit(n, cont);
    h = hmix(h, c.x);
    h = hmix(h, c.y);
    h = hmix(h, c.z);
    h = hmix(h, c.w);
    return hfinal(h);
}

// General probe: payload = w[start, end) of a byte buffer (any length).
__device__ __forceinline__ int probe_general(const DevTok &T, const uint8_t *w, int start, int end, uint32_t cont) {
    const uint32_t n = (uint32_t)(end - start);
    uint32_t h = hinit(n, cont);
    W16 first{0, 0, 0, 0};
    uint32_t b0 = 0;
    do {
        uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
        for (uint32_t k = 0; k < 16 && b0 + k < n; ++k) {
            const uint32_t v = (uint32_t)w[start + b0 + k] << (8 * (k & 3));
            if (k < 4) c0 |= v; else if (k < 8) c1 |= v; else if (k < 12) c2 |= v; else c3 |= v;
        }
        if (b0 == 0) first = W16{c0, c1, c2, c3};
        h = hmix(h, c0);
        h = hmix(h, c1);
        h = hmix(h, c2);
        h = hmix(h, c3);
        b0 += 16;
    } while (b0 < n);
    h = hfinal(h);
    const uint32_t key = n | (cont << 8);
    const Probe P = probe_load(T, h);
    for (int which = 0; which < 2; ++which) {
        const uint4 a = which ? P.a2 : P.a1, b = which ? P.b2 : P.b1;
        if (!slot_match(a, b, key, first)) continue;
        bool ok = true;
        for (uint32_t k = 16; k < n && ok; ++k) ok = T.vpool[a.z + k] == w[start + k];
        if (ok) return (int32_t)a.y;
    }
    return -1;
}

// byte k (dynamic, 0..15) of a 16-byte register word
__device__ __forceinline__ uint32_t w16_byte(const W16 &w, int k) {
    const int q = k >> 2;
    const uint32_t x = q == 0 ? w.x : q == 1 ? w.y : q == 2 ? w.z : w.w;
    return (x >> (8 * (k & 3))) & 0xFFu;
}
__device__ __forceinline__ void w16_put(W16 &w, int k, uint32_t b) {
    const int q = k >> 2;
    const uint32_t v = b << (8 * (k & 3));
    w.x |= q == 0 ? v : 0u;
    w.y |= q == 1 ? v : 0u;
    w.z |= q == 2 ? v : 0u;
    w.w |= q == 3 ? v : 0u;
}
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 load16(const uint8_t *text, int64_t p, int64_t N) {
    if (p >= 0 && p + 16 <= N) {
        const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(text + p));
        return make_uint4(x.x, x.y, x.z, x.w);
    }
    uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
    for (int k = 0; k < 16; ++k) {
        if (p + k < 0 || p + k >= N) continue;
        const uint32_t v = (uint32_t)text[p + k] << (8 * (k & 3));
        if (k < 4) w0 |= v; else if (k < 8) w1 |= v; else if (k < 12) w2 |= v; else w3 |= v;
    }
    return make_uint4(w0, w1, w2, w3);
}

}  // namespace
}  // namespace sdl
