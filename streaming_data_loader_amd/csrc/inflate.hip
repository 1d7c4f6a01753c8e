// inflate.hip -- the Provider's gzip inflate on the device.
//
// Replaces the GzipDecoder that feeds the provider's lines
// (gzip_file_provider.rs:13-28: async-compression 0.3.14 over flate2 1.0.24 /
// miniz_oxide 0.5.4, rust/Cargo.lock).  Input: gzip members (RFC 1952) back to
// back in device memory with their byte ranges; output: every member's bytes
// back to back in one device arena -- the JSON lines sdl_json_text_device reads.
//
//   k_gz_size   lane per member: header magic, ISIZE from the trailer (sizes the
//               output before anything is decoded)
//   k_inflate   one wave per member.  DEFLATE (RFC 1951) is a serial bit stream:
//               lane 0 decodes Huffman tokens through 10-bit (lit/len) and
//               8-bit (dist) LDS tables built by the whole wave per block, and
//               emits literals and (length, distance) records into an LDS batch;
//               the wave then expands the matches and resolves them by pointer
//               jumping (a byte copied from an earlier byte of the same batch
//               follows that byte's own source, so overlapping copies resolve in
//               log(depth) rounds) and stores the batch.  Compressed bytes are
//               staged in LDS 2 KiB at a time by 16-B loads of all lanes.
//   k_gz_crc    one wave per member: CRC-32 of 64 lane segments (LDS table),
//               folded with crc32_combine's x^(8n) mod P shift, against the
//               trailer's CRC.
//
// The arithmetic is RFC 1951/1952 as zlib's inflate implements it (the same
// error cases: over-subscribed or incomplete codes, missing end-of-block code,
// too many length/distance symbols, bad repeats, invalid codes, distances too
// far back, stored-length mismatch, header CRC, trailer CRC and ISIZE).  Decoding
// is fully specified by the RFC, so any conforming decoder's output -- the
// reference's miniz_oxide included -- is byte-identical; tests check against
// CPython's zlib.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

namespace sdl {
namespace {

constexpr int LB = 10, DB = 8;     // primary table bits: lit/len, dist
constexpr int IN_STAGE = 2048;     // staged compressed bytes per wave
constexpr int OBUF = 2048;         // output batch bytes
constexpr int MLCAP = 256;         // matches per batch
constexpr int HDR_ROOM = 640;      // a block header (<= ~600 B) fits in this many staged bytes
constexpr int NSYM = 320;          // lit/len (<= 288) + dist (<= 32) code lengths
constexpr uint32_t POLY = 0xEDB88320u;

enum : uint32_t { K_LIT = 0, K_LEN = 1, K_EOB = 2, K_SLOW = 3 };

__constant__ uint16_t c_len_base[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                        31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_len_extra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t c_dist_base[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                         193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dist_extra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t c_cl_order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// table entry: bits 0-3 code length (0: invalid code), 4-5 kind, 8-11 extra
// bits, 16-31 value (literal byte / length base / distance base)
__device__ __forceinline__ uint32_t sym_entry(int t, int s, int n) {
    if (t == 0) {
        if (s < 256) return (uint32_t)n | K_LIT << 4 | (uint32_t)s << 16;
        if (s == 256) return (uint32_t)n | K_EOB << 4;
        if (s < 286) return (uint32_t)n | K_LEN << 4 | (uint32_t)c_len_extra[s - 257] << 8 | (uint32_t)c_len_base[s - 257] << 16;
        return 0;  // 286, 287: invalid literal/length code
    }
    if (s < 30) return (uint32_t)n | K_LEN << 4 | (uint32_t)c_dist_extra[s] << 8 | (uint32_t)c_dist_base[s] << 16;
    return 0;  // 30, 31: invalid distance code
}

// canonical decode of a code longer than the primary table (puff's decode()):
// needs >= 15 bits in bb
__device__ uint32_t slow_decode(uint64_t bb, const uint16_t *cnt, const uint16_t *syms, int t) {
    int code = 0, first = 0, index = 0;
    for (int len = 1; len <= 15; ++len) {
        code |= (int)((bb >> (len - 1)) & 1u);
        const int count = cnt[len];
        if (code - first < count) return sym_entry(t, syms[index + code - first], len);
        index += count;
        first = (first + count) << 1;
        code <<= 1;
    }
    return 0;
}

__device__ __forceinline__ uint32_t bfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// zlib's multmodp: a(x) b(x) mod P(x), reflected
__device__ uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = b & 1u ? (b >> 1) ^ POLY : b >> 1;
    }
    return p;
}
// x^(n 2^k) mod P(x)
__device__ uint32_t x2nmodp(uint64_t n, int k, const X2N &x2n) {
    uint32_t p = 1u << 31;
    while (n) {
        if (n & 1) p = multmodp(x2n.t[k & 31], p);
        n >>= 1;
        ++k;
    }
    return p;
}

}  // namespace

// ---- lane per member: header magic + ISIZE ------------------------------------
__global__ void k_gz_size(const uint8_t *__restrict__ in, uint64_t in_len, const uint64_t *__restrict__ moff, uint64_t n,
                          uint32_t *__restrict__ size, int32_t *__restrict__ status, unsigned long long *__restrict__ total) {
    const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= n) return;
    const uint64_t a = moff[m], z = moff[m + 1];
    int32_t st = GZ_OK;
    uint32_t sz = 0;
    if (a > z || z > in_len) st = GZ_E_RANGE;
    else if (z - a < 18) st = GZ_E_TRUNC;
    else if (in[a] != 0x1f || in[a + 1] != 0x8b || in[a + 2] != 8) st = GZ_E_HEADER;
    else {
        sz = (uint32_t)in[z - 4] | (uint32_t)in[z - 3] << 8 | (uint32_t)in[z - 2] << 16 | (uint32_t)in[z - 1] << 24;
        // DEFLATE expands at most 1032:1 (258-byte copies in 2 bits): a larger ISIZE is corrupt,
        // and must not size the arena
        if ((uint64_t)sz > 1032 * (z - a) + 64) {
            st = GZ_E_SIZE;
            sz = 0;
        }
    }
    size[m] = sz;
    status[m] = st;
    if (sz) atomicAdd(total, (unsigned long long)sz);
}

// ---- one wave per member --------------------------------------------------------
__global__ __launch_bounds__(64) void k_inflate(const uint8_t *__restrict__ in, const uint64_t *__restrict__ moff,
                                               uint64_t n, const uint32_t *__restrict__ ooff, uint8_t *__restrict__ out,
                                               int32_t *__restrict__ status, uint32_t *__restrict__ tcrc) {
    __shared__ uint32_t s_lit[1 << LB], s_dst[1 << DB];
    __shared__ uint16_t s_cnt[2][16];
    __shared__ uint16_t s_sym[NSYM];     // symbols sorted by code: lit/len [0, 288), dist [288, 320)
    __shared__ uint16_t s_rc[NSYM];      // bit-reversed canonical code per symbol
    __shared__ uint8_t s_len[NSYM + 32];  // code lengths (lit/len, then dist); code-length code at NSYM..
    __shared__ __attribute__((aligned(16))) uint8_t s_in[IN_STAGE + 16];
    __shared__ uint8_t s_ob[OBUF];
    __shared__ uint16_t s_ref[OBUF];     // 0: byte known; d: byte equals the one d back
    __shared__ uint32_t s_mpl[MLCAP];    // match: batch offset | length << 16
    __shared__ uint16_t s_md[MLCAP];     // match distance

    const uint64_t m = blockIdx.x;
    const int lane = (int)threadIdx.x;
    if (status[m] != GZ_OK) return;  // sizing found the member unusable
    const uint64_t ma = moff[m], mz = moff[m + 1];
    uint8_t *const dst = out + ooff[m];
    const uint32_t cap = ooff[m + 1] - ooff[m];
    const uint32_t mlen = (uint32_t)(mz - ma);
    typedef __attribute__((address_space(3))) uint32_t lds_w;
    const lds_w *in32 = (const lds_w *)s_in;

    // lane 0's decoder state (other lanes' copies unused)
    uint64_t bb = 0;
    int bc = 0, ip = 0;
    int32_t err = GZ_OK;
    bool in_block = false, final_seen = false;
    uint32_t nb = 0, nm = 0;
    auto need = [&](int k) {  // byte refill to >= k bits (k <= 57)
        while (bc < k) {
            bb |= (uint64_t)s_in[ip++] << bc;
            bc += 8;
        }
    };
    auto drop = [&](int k) {
        bb >>= k;
        bc -= k;
    };

    // ---- header (lane 0, straight from global memory) ----
    uint32_t p = 10;  // member-relative
    if (lane == 0) {
        const uint32_t flg = in[ma + 3];
        if (flg & 0xE0u) err = GZ_E_HEADER;  // reserved flag bits (zlib: "unknown header flags set")
        if (!err && (flg & 4u)) {  // FEXTRA
            if (p + 2 > mlen) err = GZ_E_TRUNC;
            else p += 2u + ((uint32_t)in[ma + p] | (uint32_t)in[ma + p + 1] << 8);
        }
        for (uint32_t f = 8; f <= 16 && !err; f <<= 1)  // FNAME, FCOMMENT: zero-terminated
            if (flg & f) {
                while (p < mlen && in[ma + p]) ++p;
                ++p;
            }
        if (!err && (flg & 2u)) {  // FHCRC: low 16 bits of the header's CRC-32
            if (p + 2 > mlen) err = GZ_E_TRUNC;
            else {
                uint32_t c = ~0u;
                for (uint32_t i = 0; i < p; ++i) {
                    c ^= in[ma + i];
                    for (int k = 0; k < 8; ++k) c = c & 1u ? (c >> 1) ^ POLY : c >> 1;
                }
                if (((~c) & 0xFFFFu) != ((uint32_t)in[ma + p] | (uint32_t)in[ma + p + 1] << 8)) err = GZ_E_HCRC;
                p += 2;
            }
        }
        if (!err && (uint64_t)p + 8 > mlen) err = GZ_E_TRUNC;
    }
    if (bfl((uint32_t)err) != GZ_OK) {
        if (lane == 0) status[m] = err;
        return;
    }

    // ---- staging of compressed bytes: s_in[0] is member byte sbase (16-B aligned in `in`) ----
    uint64_t sbase = 0;  // absolute
    auto restage = [&](uint64_t abs) {
        sbase = abs & ~(uint64_t)15;
#pragma unroll
        for (int k = 0; k < IN_STAGE / 16 / 64; ++k) {
            const int o = 16 * (lane + 64 * k);
            const uint64_t q = sbase + (uint64_t)o;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (q + 16 <= mz) {
                v = *reinterpret_cast<const uint4 *>(in + q);
            } else if (q < mz) {
                uint32_t w[4] = {0, 0, 0, 0};
                for (int b = 0; b < 16 && q + b < mz; ++b) w[b >> 2] |= (uint32_t)in[q + b] << (8 * (b & 3));
                v = make_uint4(w[0], w[1], w[2], w[3]);
            }
            *reinterpret_cast<uint4 *>(s_in + o) = v;
        }
        if (lane == 0) *reinterpret_cast<uint4 *>(s_in + IN_STAGE) = make_uint4(0, 0, 0, 0);
        __syncthreads();
        if (lane == 0) ip = (int)(abs - sbase);
    };
    restage(ma + bfl(p));

    enum : uint32_t { A_DONE, A_ERR, A_RESTAGE, A_BUILD, A_FLUSH, A_STORED };
    uint32_t produced = 0;  // wave-uniform
    for (;;) {
        uint32_t act = A_DONE, x0 = 0, x1 = 0;
        if (lane == 0) {
            if (!in_block) {
                if (final_seen) act = A_DONE;
                else if (ip > IN_STAGE - HDR_ROOM) act = A_RESTAGE;
                else {
                    need(3);
                    final_seen = bb & 1u;
                    const uint32_t type = (uint32_t)(bb >> 1) & 3u;
                    drop(3);
                    if (type == 0) {  // stored
                        drop(bc & 7);
                        need(32);
                        const uint32_t len = (uint32_t)bb & 0xFFFFu, nlen = (uint32_t)(bb >> 16) & 0xFFFFu;
                        drop(32);
                        if (len != (~nlen & 0xFFFFu)) {
                            err = GZ_E_STORED;
                            act = A_ERR;
                        } else {
                            act = A_STORED;
                            x0 = (uint32_t)(sbase + (uint64_t)ip - (uint64_t)(bc >> 3) - ma);  // data start
                            x1 = len;
                            bb = 0;
                            bc = 0;
                        }
                    } else if (type == 1) {  // fixed codes
                        for (int s = 0; s < 288; ++s) s_len[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
                        for (int s = 0; s < 32; ++s) s_len[288 + s] = 5;
                        act = A_BUILD;
                        x0 = 288;
                        x1 = 32 | 1u << 16;
                    } else if (type == 2) {  // dynamic codes
                        need(14);
                        const int hlit = (int)(bb & 31u) + 257, hdist = (int)((bb >> 5) & 31u) + 1,
                                  hclen = (int)((bb >> 10) & 15u) + 4;
                        drop(14);
                        if (hlit > 286 || hdist > 30) err = GZ_E_CODES;
                        uint8_t *cl = s_len + NSYM;
                        for (int i = 0; i < 19; ++i) cl[i] = 0;
                        for (int i = 0; i < hclen && !err; ++i) {
                            need(3);
                            cl[c_cl_order[i]] = (uint8_t)(bb & 7u);
                            drop(3);
                        }
                        // code-length code: complete, <= 7 bits; its 128-entry table in s_dst
                        uint16_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0}, next[8];
                        for (int i = 0; i < 19; ++i) ++cnt[cl[i]];
                        int left = 1;
                        for (int l = 1; l < 8; ++l) left = (left << 1) - cnt[l];
                        if (!err && left != 0) err = GZ_E_CODES;  // over-subscribed or incomplete (or empty)
                        if (!err) {
                            uint32_t code = 0;
                            cnt[0] = 0;
                            for (int l = 1; l < 8; ++l) {
                                code = (code + cnt[l - 1]) << 1;
                                next[l] = (uint16_t)code;
                            }
                            for (int s = 0; s < 19; ++s)
                                if (cl[s]) {
                                    const int l = cl[s];
                                    const uint32_t r = __builtin_bitreverse32((uint32_t)next[l]++) >> (32 - l);
                                    for (uint32_t i = r; i < 128; i += 1u << l) s_dst[i] = (uint32_t)l | (uint32_t)s << 16;
                                }
                            const int total = hlit + hdist;
                            int i = 0;
                            while (i < total && !err) {
                                need(14);
                                const uint32_t e = s_dst[bb & 127u];
                                const int sym = (int)(e >> 16);
                                drop((int)(e & 15u));
                                if (sym < 16) {
                                    s_len[i++] = (uint8_t)sym;
                                    continue;
                                }
                                int rep;
                                uint8_t v = 0;
                                if (sym == 16) {
                                    if (i == 0) { err = GZ_E_CODES; break; }
                                    v = s_len[i - 1];
                                    rep = 3 + (int)(bb & 3u);
                                    drop(2);
                                } else if (sym == 17) {
                                    rep = 3 + (int)(bb & 7u);
                                    drop(3);
                                } else {
                                    rep = 11 + (int)(bb & 127u);
                                    drop(7);
                                }
                                if (i + rep > total) { err = GZ_E_CODES; break; }
                                while (rep--) s_len[i++] = v;
                            }
                            if (!err && s_len[256] == 0) err = GZ_E_CODES;  // missing end-of-block code
                        }
                        if (err) act = A_ERR;
                        else {
                            act = A_BUILD;
                            x0 = (uint32_t)hlit;
                            x1 = (uint32_t)hdist;
                        }
                    } else {
                        err = GZ_E_BTYPE;
                        act = A_ERR;
                    }
                }
            } else {
                // ---- Huffman tokens into the batch ----
                bool eob = false, rs = false;
                for (;;) {
                    if (nb > (uint32_t)(OBUF - 259) || nm >= (uint32_t)MLCAP) break;
                    if (ip > IN_STAGE - 16) { rs = true; break; }
                    if (bc <= 32) {
                        const int a = ip >> 2;
                        const uint32_t w = __builtin_amdgcn_alignbyte(in32[a + 1], in32[a], (uint32_t)(ip & 3));
                        bb |= (uint64_t)w << bc;
                        ip += 4;
                        bc += 32;
                    }
                    uint32_t e = s_lit[bb & ((1u << LB) - 1u)];
                    if (((e >> 4) & 3u) == K_SLOW) e = slow_decode(bb, s_cnt[0], s_sym, 0);
                    const int nbits = (int)(e & 15u);
                    if (nbits == 0) { err = GZ_E_CODE; break; }
                    drop(nbits);
                    const uint32_t kind = (e >> 4) & 3u;
                    if (kind == K_LIT) {
                        if (produced + nb >= cap) { err = GZ_E_OVER; break; }
                        s_ob[nb] = (uint8_t)(e >> 16);
                        s_ref[nb] = 0;
                        ++nb;
                        continue;
                    }
                    if (kind == K_EOB) { eob = true; break; }
                    const int eb = (int)((e >> 8) & 15u);
                    const uint32_t len = (e >> 16) + ((uint32_t)bb & ((1u << eb) - 1u));
                    drop(eb);
                    if (bc <= 32) {
                        const int a = ip >> 2;
                        const uint32_t w = __builtin_amdgcn_alignbyte(in32[a + 1], in32[a], (uint32_t)(ip & 3));
                        bb |= (uint64_t)w << bc;
                        ip += 4;
                        bc += 32;
                    }
                    uint32_t d = s_dst[bb & ((1u << DB) - 1u)];
                    if (((d >> 4) & 3u) == K_SLOW) d = slow_decode(bb, s_cnt[1], s_sym + 288, 1);
                    const int dbits = (int)(d & 15u);
                    if (dbits == 0) { err = GZ_E_CODE; break; }
                    drop(dbits);
                    const int db = (int)((d >> 8) & 15u);
                    const uint32_t dist = (d >> 16) + ((uint32_t)bb & ((1u << db) - 1u));
                    drop(db);
                    if (dist > produced + nb) { err = GZ_E_FAR; break; }
                    if (produced + nb + len > cap) { err = GZ_E_OVER; break; }
                    s_mpl[nm] = nb | len << 16;
                    s_md[nm] = (uint16_t)dist;
                    ++nm;
                    nb += len;
                }
                if (err) act = A_ERR;
                else {
                    act = A_FLUSH;
                    x0 = nb;
                    x1 = nm | (eob ? 1u << 16 : 0u) | (rs ? 1u << 17 : 0u);
                    if (eob) in_block = false;
                    // input consumed past the member: truncated
                    if (sbase + (uint64_t)ip - (uint64_t)(bc >> 3) > mz) {
                        err = GZ_E_TRUNC;
                        act = A_ERR;
                    }
                }
            }
        }
        act = bfl(act);
        x0 = bfl(x0);
        x1 = bfl(x1);
        if (act == A_DONE || act == A_ERR) break;
        if (act == A_RESTAGE) {
            const uint64_t abs = (uint64_t)bfl((uint32_t)(sbase + (uint64_t)ip - ma)) + ma;
            restage(abs);
            continue;
        }
        if (act == A_BUILD) {
            // canonical codes (lane 0), then the primary tables (all lanes)
            const int nl = (int)x0, nd = (int)(x1 & 0xFFFFu);
            const bool fixed = (x1 >> 16) & 1u;
            if (lane == 0) {
                for (int t = 0; t < 2 && !err; ++t) {
                    const int base = t ? nl : 0, cntn = t ? nd : nl;
                    uint16_t cnt[16], next[16];
                    for (int l = 0; l < 16; ++l) cnt[l] = 0;
                    for (int s = 0; s < cntn; ++s) ++cnt[s_len[base + s]];
                    cnt[0] = 0;
                    int left = 1, mx = 0;
                    for (int l = 1; l < 16; ++l) {
                        left = (left << 1) - cnt[l];
                        if (left < 0) break;
                        if (cnt[l]) mx = l;
                    }
                    // over-subscribed; incomplete unless a single 1-bit code (zlib's inflate_table)
                    if (!fixed && (left < 0 || (mx > 0 && left > 0 && mx != 1))) err = GZ_E_CODES;
                    uint32_t code = 0, off = 0;
                    uint16_t offs[16];
                    for (int l = 1; l < 16; ++l) {
                        code = (code + cnt[l - 1]) << 1;
                        next[l] = (uint16_t)code;
                        offs[l] = (uint16_t)off;
                        off += cnt[l];
                    }
                    uint16_t *syms = s_sym + (t ? 288 : 0);
                    for (int s = 0; s < cntn; ++s) {
                        const int l = s_len[base + s];
                        if (!l) continue;
                        s_rc[base + s] = (uint16_t)(__builtin_bitreverse32((uint32_t)next[l]++) >> (32 - l));
                        syms[offs[l]++] = (uint16_t)s;
                    }
                    for (int l = 0; l < 16; ++l) s_cnt[t][l] = cnt[l];
                }
                if (!err) in_block = true;
            }
            if (bfl((uint32_t)err) != GZ_OK) break;
            for (int i = lane; i < (1 << LB); i += 64) s_lit[i] = 0;
            for (int i = lane; i < (1 << DB); i += 64) s_dst[i] = 0;
            __syncthreads();
            for (int s = lane; s < nl + nd; s += 64) {
                const int t = s < nl ? 0 : 1, sym = t ? s - nl : s, l = s_len[s];
                if (!l) continue;
                const int bits = t ? DB : LB;
                uint32_t *tab = t ? s_dst : s_lit;
                const uint32_t r = s_rc[s];
                if (l <= bits) {
                    const uint32_t e = sym_entry(t, sym, l);
                    if (e)
                        for (uint32_t i = r; i < (1u << bits); i += 1u << l) tab[i] = e;
                } else {
                    tab[r & ((1u << bits) - 1u)] = K_SLOW << 4;
                }
            }
            __syncthreads();
            continue;
        }
        if (act == A_STORED) {
            const uint32_t start = x0, len = x1;
            int32_t e2 = GZ_OK;
            if ((uint64_t)start + len + 8 > mlen) e2 = GZ_E_TRUNC;
            else if (produced + len > cap) e2 = GZ_E_OVER;
            if (e2 != GZ_OK) {
                if (lane == 0) err = e2;
                break;
            }
            for (uint32_t i = (uint32_t)lane; i < len; i += 64) dst[produced + i] = in[ma + start + i];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            produced += len;
            restage(ma + start + len);
            continue;
        }
        // ---- A_FLUSH: expand the matches, resolve them, store the batch ----
        const uint32_t fnb = x0, fnm = x1 & 0xFFFFu;
        __syncthreads();  // lane 0's batch and match list
        for (uint32_t k = (uint32_t)lane; k < fnm; k += 64) {
            const uint32_t pl = s_mpl[k], pos = pl & 0xFFFFu, len = pl >> 16;
            const uint16_t d = s_md[k];
            for (uint32_t i = 0; i < len; ++i) s_ref[pos + i] = d;
        }
        __syncthreads();
        if (fnm) {
            for (;;) {
                bool more = false;
                for (uint32_t q = (uint32_t)lane; q < fnb; q += 64) {
                    const uint32_t d = s_ref[q];
                    if (!d) continue;
                    const int src = (int)q - (int)d;
                    uint32_t v;
                    if (src < 0) {
                        v = dst[(int64_t)produced + src];  // history: an earlier batch (distance checked)
                    } else {
                        const uint32_t d2 = s_ref[src];
                        if (d2) {  // the source is itself a copy: follow it
                            s_ref[q] = (uint16_t)(d + d2);
                            more = true;
                            continue;
                        }
                        v = s_ob[src];
                    }
                    s_ob[q] = (uint8_t)v;
                    s_ref[q] = 0;
                }
                __syncthreads();
                if (!__any(more)) break;
            }
        }
        for (uint32_t q = (uint32_t)lane; q < fnb; q += 64) dst[produced + q] = s_ob[q];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        __syncthreads();
        produced += fnb;
        if (lane == 0) {
            nb = 0;
            nm = 0;
        }
        if ((x1 >> 17) & 1u) {
            const uint64_t abs = (uint64_t)bfl((uint32_t)(sbase + (uint64_t)ip - ma)) + ma;
            restage(abs);
        }
    }
    // ---- trailer ----
    if (lane == 0) {
        if (!err) {
            drop(bc & 7);
            const uint64_t t = sbase + (uint64_t)ip - (uint64_t)(bc >> 3);  // absolute
            if (t + 8 > mz) err = GZ_E_TRUNC;
            else if (t + 8 != mz) err = GZ_E_TRAIL;  // bytes after the member's trailer
            else {
                const uint32_t crc = (uint32_t)in[t] | (uint32_t)in[t + 1] << 8 | (uint32_t)in[t + 2] << 16 |
                                     (uint32_t)in[t + 3] << 24;
                const uint32_t isz = (uint32_t)in[t + 4] | (uint32_t)in[t + 5] << 8 | (uint32_t)in[t + 6] << 16 |
                                     (uint32_t)in[t + 7] << 24;
                if (isz != produced || produced != cap) err = GZ_E_SIZE;
                tcrc[m] = crc;
            }
        }
        status[m] = err;
    }
}

// ---- one wave per member: CRC-32 of the output against the trailer ---------------
__global__ __launch_bounds__(64) void k_gz_crc(const uint32_t *__restrict__ ooff, const uint8_t *__restrict__ out,
                                              uint64_t n, const uint32_t *__restrict__ tcrc, X2N x2n,
                                              int32_t *__restrict__ status, uint32_t *__restrict__ bad) {
    __shared__ uint32_t T[256];
    __shared__ uint32_t s_p[64];
    const uint64_t m = blockIdx.x;
    const int lane = (int)threadIdx.x;
    for (int i = lane; i < 256; i += 64) {
        uint32_t c = (uint32_t)i;
        for (int k = 0; k < 8; ++k) c = c & 1u ? (c >> 1) ^ POLY : c >> 1;
        T[i] = c;
    }
    __syncthreads();
    if (status[m] == GZ_OK) {
        const uint32_t a = ooff[m], len = ooff[m + 1] - a;
        const uint32_t seg = ((len + 63u) / 64u + 15u) & ~15u;
        const uint32_t la = (uint32_t)lane * seg < len ? (uint32_t)lane * seg : len;
        const uint32_t lz = la + seg < len ? la + seg : len;
        const uint8_t *src = out + a;
        uint32_t c = ~0u;
        uint32_t i = la;
        for (; i + 4 <= lz; i += 4) {
            const uint32_t b0 = src[i], b1 = src[i + 1], b2 = src[i + 2], b3 = src[i + 3];
            c = T[(c ^ b0) & 255u] ^ (c >> 8);
            c = T[(c ^ b1) & 255u] ^ (c >> 8);
            c = T[(c ^ b2) & 255u] ^ (c >> 8);
            c = T[(c ^ b3) & 255u] ^ (c >> 8);
        }
        for (; i < lz; ++i) c = T[(c ^ src[i]) & 255u] ^ (c >> 8);
        s_p[lane] = ~c;
        __syncthreads();
        if (lane == 0) {
            // crc32_combine over the lanes' segments: crc(A B) = crc(A) x^(8|B|) mod P ^ crc(B)
            const uint32_t xs = x2nmodp(seg, 3, x2n);
            uint32_t tot = s_p[0];
            for (int l = 1; l < 64; ++l) {
                const uint32_t sa = (uint32_t)l * seg;
                if (sa >= len) break;
                const uint32_t sl = sa + seg <= len ? seg : len - sa;
                tot = multmodp(sl == seg ? xs : x2nmodp(sl, 3, x2n), tot) ^ s_p[l];
            }
            if (len == 0) tot = 0;
            if (tot != tcrc[m]) status[m] = GZ_E_CRC;
        }
    }
    __syncthreads();
    if (lane == 0 && status[m] != GZ_OK) {
        atomicAdd(&bad[0], 1u);
        atomicMin(&bad[1], (uint32_t)m);
    }
}

hipError_t launch_gz_size(const uint8_t *in, uint64_t in_len, const uint64_t *moff, uint64_t n, uint32_t *size,
                          int32_t *status, unsigned long long *total, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_gz_size, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, in, in_len, moff, n, size, status,
                       total);
    return hipGetLastError();
}

hipError_t launch_inflate(const uint8_t *in, const uint64_t *moff, uint64_t n, const uint32_t *ooff, uint8_t *out,
                          int32_t *status, uint32_t *tcrc, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_inflate, dim3((unsigned)n), dim3(64), 0, st, in, moff, n, ooff, out, status, tcrc);
    return hipGetLastError();
}

hipError_t launch_gz_crc(const uint32_t *ooff, const uint8_t *out, uint64_t n, const uint32_t *tcrc, const X2N &x2n,
                         int32_t *status, uint32_t *bad, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_gz_crc, dim3((unsigned)n), dim3(64), 0, st, ooff, out, n, tcrc, x2n, status, bad);
    return hipGetLastError();
}

}  // namespace sdl
