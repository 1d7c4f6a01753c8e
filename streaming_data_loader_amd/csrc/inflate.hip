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
//               10-bit (dist) LDS tables built by the whole wave per block, and
//               emits literals and (length, distance) records into an LDS batch;
//               the wave then expands the matches and resolves them by pointer
//               jumping (a byte copied from an earlier byte of the same batch
//               follows that byte's own source, so overlapping copies resolve in
//               log(depth) rounds) and stores the batch.  Compressed bytes are
//               staged in LDS 1 KiB at a time by 16-B loads of all lanes.
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
#include <cstdio>
#include <type_traits>

#include "device_util.hpp"
#include "kernels.hpp"

namespace sdl {
namespace {

constexpr int LB = 10, DB = 10;    // primary table bits: lit/len, dist (long_decode covers 11..15)
#ifndef SDL_GZ_OBUF
#define SDL_GZ_OBUF 512
#endif
constexpr int IN_STAGE = 1024;  // staged compressed bytes per wave
constexpr int OBUF = SDL_GZ_OBUF;       // output batch bytes
constexpr int MLCAP = OBUF / 8;         // matches per batch
#ifndef SDL_GZ_ALLOW_SMALL_OBUF  // (diagnostic builds only: exercises the no-progress exit below)
static_assert(OBUF >= 512, "a batch must take any 258-byte match (else an empty batch never fills: no progress)");
#endif
constexpr int HDR_ROOM = 640;      // a block header (<= ~600 B) fits in this many staged bytes
constexpr int NSYM = 320;          // lit/len (<= 288) + dist (<= 32) code lengths
constexpr uint32_t POLY = 0xEDB88320u;

enum : uint32_t { K_LIT = 0, K_LEN = 1, K_EOB = 2, K_SLOW = 3 };
constexpr uint32_t K_BAD = 3;  // (token kinds: K_SLOW never names a decoded token)

__constant__ uint16_t c_len_base[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                        31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_len_extra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t c_dist_base[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                         193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dist_extra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t c_cl_order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// table entry: bits 0-3 code length (0: no such code), 4-5 kind, 8-11 extra
// bits, 16-31 value (literal byte / length base / distance base).  The symbols
// a code may name but DEFLATE does not define (lit/len 286, 287; distance 30,
// 31) keep their code length with extra = 15 (no real symbol has that many),
// so a decoder knows how many bits zlib reads before it rejects them.
constexpr uint32_t X_BADSYM = 15u;
__device__ __forceinline__ uint32_t sym_entry(int t, int s, int n) {
    if (t == 0) {
        if (s < 256) return (uint32_t)n | K_LIT << 4 | (uint32_t)s << 16;
        if (s == 256) return (uint32_t)n | K_EOB << 4;
        if (s < 286) return (uint32_t)n | K_LEN << 4 | (uint32_t)c_len_extra[s - 257] << 8 | (uint32_t)c_len_base[s - 257] << 16;
        return (uint32_t)n | K_LEN << 4 | X_BADSYM << 8;  // 286, 287: invalid literal/length symbol
    }
    if (s < 30) return (uint32_t)n | K_LEN << 4 | (uint32_t)c_dist_extra[s] << 8 | (uint32_t)c_dist_base[s] << 16;
    return (uint32_t)n | K_LEN << 4 | X_BADSYM << 8;  // 30, 31: invalid distance symbol
}

// A code longer than the primary table (11..15 bits): canonical decode by
// limits.  c = the next 15 stream bits, first bit most significant; the code
// has length L for the smallest L with c < lim[L - 11] (lim = one past the
// last code of length L, left-aligned to 15 bits); its symbol is sorted entry
// base[L - 11] + (c >> (15 - L)).  All lanes can do this (one LDS load).
__device__ __forceinline__ uint32_t long_decode(uint64_t bits, const uint32_t *lim, const uint32_t *base,
                                                const uint32_t *sent) {
    const uint32_t c = __builtin_bitreverse32((uint32_t)bits) >> 17;
    uint32_t idx = ~0u;
#pragma unroll
    for (int i = 4; i >= 0; --i)
        if (c < lim[i]) idx = base[i] + (c >> (4 - i));
    return idx == ~0u ? 0u : sent[idx];
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

// Diagnostic build (-DSDL_STAMPS): lane 0 of every wave adds the s_memtime
// cycles of each phase and event counts; never in the product.
#ifdef SDL_STAMPS
__device__ unsigned long long sdl_gz_cycles[8], sdl_gz_counts[8];
#define GZ_STAMP(k)                                                       \
    do {                                                                  \
        if (threadIdx.x == 0) {                                           \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();  \
            atomicAdd(&sdl_gz_cycles[k], t_ - gz_prev_);                  \
            gz_prev_ = t_;                                                \
        }                                                                 \
    } while (0)
#define GZ_COUNT(k) do { if (threadIdx.x == 0) atomicAdd(&sdl_gz_counts[k], 1ull); } while (0)
void print_gz_cycles() {
    unsigned long long h[8], c[8];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(sdl_gz_cycles), sizeof(h)) != hipSuccess) return;
    if (hipMemcpyFromSymbol(c, HIP_SYMBOL(sdl_gz_counts), sizeof(c)) != hipSuccess) return;
    static const char *names[] = {"header+stage", "block hdr+emit", "tables", "token decode", "expand", "resolve", "store", "walk"};
    unsigned long long tot = 0;
    for (int i = 0; i < 8; ++i) tot += h[i];
    for (int i = 0; i < 8; ++i)
        fprintf(stderr, "[gz stamps] %-14s %6.2f%%  count %llu  cycles/count %.0f\n", names[i],
                tot ? 100.0 * (double)h[i] / (double)tot : 0.0, c[i], c[i] ? (double)h[i] / (double)c[i] : 0.0);
}
#else
#define GZ_STAMP(k) do {} while (0)
#define GZ_COUNT(k) do {} while (0)
#endif

// ---- lane per member: header magic + ISIZE ------------------------------------
__global__ void k_gz_size(const uint8_t *__restrict__ in, uint64_t in_len, const uint64_t *__restrict__ moff, uint64_t n,
                          uint32_t *__restrict__ size, int32_t *__restrict__ status, unsigned long long *__restrict__ total,
                          const uint64_t *__restrict__ mend) {
    const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= n) return;
    const uint64_t a = moff[m], z = mend ? mend[m] : moff[m + 1];
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
// Tokens are decoded speculatively by all lanes: lane i decodes the token that
// would start at bit bp + i (lit/len code, length extra bits, distance code and
// extra bits: <= 48 bits from a 64-bit window of the staged input), and the
// scalar unit walks the real chain from bit bp through the lanes' token lengths
// (v_readlane), so one pass settles every token starting in the next 64 bits.
// Literals and match records then go to the LDS batch in parallel (positions
// by a wave prefix sum of the tokens' output lengths).
//
// CH (chunked members, see kernels.hpp): a wave decodes one chunk of a large
// member -- from its start bit (or the member header) to the first block
// boundary at or past its stop bit -- into a 16-bit slot: a byte, or 256 + w for
// a copy from byte w of the 32 KiB window before the chunk (resolved later, in
// stream order).  A block that would overflow the slot ends the chunk at that
// block's start (GZC_SOFT) unless it is the chunk's first.
template <bool CH>
__global__ __launch_bounds__(64) void k_inflate_t(const uint8_t *__restrict__ in, const uint64_t *__restrict__ moff,
                                                 uint64_t n, const uint32_t *__restrict__ ooff, uint8_t *__restrict__ out,
                                                 int32_t *__restrict__ status, uint32_t *__restrict__ tcrc,
                                                 GzChunkArgs ca) {
    typedef typename std::conditional<CH, uint16_t, uint8_t>::type OT;  // batch / output values
    __shared__ uint32_t s_lit[1 << LB], s_dst[1 << DB];
    __shared__ uint32_t s_sent[NSYM];     // table entries of the symbols sorted by code: lit/len [0, 288), dist [288, 320)
    __shared__ uint8_t s_len[NSYM + 32];  // code lengths (lit/len, then dist); code-length code at NSYM..
    __shared__ __attribute__((aligned(16))) uint32_t s_in32[IN_STAGE / 4 + 4];
    __shared__ OT s_ob[OBUF];
    __shared__ uint16_t s_ref[OBUF];      // 0: byte known; d: byte equals the one d back
    __shared__ uint32_t s_mpl[MLCAP];     // match: batch offset | length << 16
    __shared__ uint16_t s_md[MLCAP];      // match distance

    const uint64_t m = blockIdx.x;
    const int lane = (int)threadIdx.x;
    uint64_t ma, mz, start_bit = GZ_START_HEADER, hdr_bit = GZ_START_HEADER;
    uint32_t tgt = 0;  // (CH) the next chunk this one may hand over to
    uint32_t cap, c = 0;
    OT *dst;
    if constexpr (CH) {
        c = ca.list[m];
        ma = ca.ma;
        mz = ca.mz;
        cap = ca.cap;
        dst = ca.slots + (uint64_t)c * ca.cap;
        start_bit = ca.start_bit[c];
        hdr_bit = ca.hdr_bit[c];
    } else {
        if (status[m] != GZ_OK) return;  // sizing found the member unusable
        ma = moff[m];
        mz = ca.mend ? ca.mend[m] : moff[m + 1];
        dst = out + ooff[m];
        cap = ooff[m + 1] - ooff[m];
    }
    const bool from_header = start_bit == GZ_START_HEADER;
    const uint32_t mlen = (uint32_t)(mz - ma);
    uint8_t *const s_in = reinterpret_cast<uint8_t *>(s_in32);
#ifdef SDL_STAMPS
    unsigned long long gz_prev_ = __builtin_amdgcn_s_memtime();
#endif

    // ---- member header (lane 0, straight from global memory) ----
    int32_t err = GZ_OK;
    uint32_t p = 10;  // member-relative
    if (lane == 0 && from_header) {
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
        if (lane == 0) {
            if constexpr (CH) ca.status[c] = err;
            else status[m] = err;
        }
        return;
    }

    // ---- staged input: s_in[0] is byte sbase (16-B aligned in `in`); bp = bit position in s_in ----
    uint64_t sbase = 0;  // wave-uniform
    uint32_t bp = 0;     // wave-uniform
    auto restage = [&](uint64_t abs, uint32_t bit) {
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
        bp = (uint32_t)(abs - sbase) * 8u + bit;
    };
    auto peek = [&](uint32_t pos) -> uint32_t {  // 32 bits from bit `pos` of the stage
        const uint32_t a = pos >> 5;
        return __builtin_amdgcn_alignbit(s_in32[a + 1], s_in32[a], pos & 31u);
    };
    // (CH) a chunk that resumes inside a block parses that block's header first
    bool resume = !from_header && hdr_bit != start_bit;  // wave-uniform
    if (from_header) restage(ma + bfl(p), 0);
    else restage(hdr_bit >> 3, (uint32_t)(hdr_bit & 7u));
    GZ_STAMP(0);
    GZ_COUNT(0);

    enum : uint32_t { A_ERR, A_BUILD, A_STORED };
    uint32_t produced = 0, nb = 0, nm = 0;  // wave-uniform
    bool in_block = false, final_seen = false;
    uint64_t blk_bit = 0;    // (CH) the current block's header bit
    // (CH) the last point the output was flushed at -- a block boundary or a batch inside a
    // block (with that block's header bit): where a chunk stops when its slot is full
    uint64_t cut_bit = start_bit, cut_hdr = hdr_bit;
    uint32_t cut_prod = 0;
    bool soft = false;       // (CH) stopped at the cut: the slot is full
    if constexpr (CH) tgt = ca.tgt0[c];
    bool handed = false;     // (CH) stopped at chunk tgt's start
    uint32_t limL[5], baseL[5], limD[5], baseD[5];  // long codes (11..15 bits) of the block, long_decode
    // Every pass consumes bits, flushes a non-empty batch or restages, so a
    // member takes fewer than 4 (8 mlen + cap) + 64 passes; the cap and the
    // explicit no-progress test below turn a decoder bug or an unforeseen
    // input into GZ_E_STALL instead of a wave that never finishes.
    const uint64_t pass_cap = 4ull * (8ull * (uint64_t)mlen + (uint64_t)cap) + 64ull;
    uint64_t passes = 0;  // wave-uniform
    for (;;) {
        if (++passes > pass_cap) {
            if (lane == 0) err = GZ_E_STALL;
            break;
        }
        if (!in_block) {
            if (final_seen) break;
            if constexpr (CH) {
                blk_bit = 8 * sbase + bp;
                if (!resume) {
                    cut_bit = cut_hdr = blk_bit;
                    cut_prod = produced;
                    // hand over to the first later chunk whose searched start is this block: a
                    // candidate behind us was no block start; a block start the search did not
                    // pick (stored, fixed, past its span) is decoded through
                    while (tgt < ca.n_chunks && blk_bit >= ca.nominal[tgt]) {
                        const uint64_t f = ca.found[tgt];
                        if (blk_bit == f) {
                            handed = true;
                            break;
                        }
                        if (blk_bit < f) break;
                        ++tgt;
                    }
                    if (handed) break;
                }
            }
            if (bp > 8u * (IN_STAGE - HDR_ROOM)) {
                restage(sbase + (bp >> 3), bp & 7u);
                continue;
            }
            // ---- block header (lane 0): a 64-bit reader refilled 32 bits at a time ----
            uint32_t act = A_ERR, x0 = 0, x1 = 0, nbp = 0, fin = 0;
            if (lane == 0) {
                uint64_t bb = 0;
                int bc = 0;
                uint32_t fill = bp;
                auto need = [&](int k) {  // k <= 32
                    if (bc < k) {
                        bb |= (uint64_t)peek(fill) << bc;
                        fill += 32;
                        bc += 32;
                    }
                };
                auto drop = [&](int k) {
                    bb >>= k;
                    bc -= k;
                };
                // the first error and the bits consumed when it was found: a reader
                // that ran past the deflate data (the trailer's 8 bytes are not
                // input) fails with GZ_E_TRUNC first, as zlib's does
                uint32_t err_bits = 0;
                auto seterr = [&](int32_t code, uint32_t at_bits) {
                    if (!err) {
                        err = code;
                        err_bits = at_bits;
                    }
                };
                need(3);
                fin = (uint32_t)bb & 1u;
                const uint32_t type = (uint32_t)(bb >> 1) & 3u;
                drop(3);
                if (type == 0) {  // stored: LEN, NLEN at the next byte boundary
                    const uint32_t at = (fill - (uint32_t)bc + 7u) & ~7u;
                    const uint32_t w = peek(at);
                    if ((w & 0xFFFFu) != (~(w >> 16) & 0xFFFFu)) seterr(GZ_E_STORED, at + 32u);
                    else if ((int64_t)at + 32 > 8 * ((int64_t)mz - 8 - (int64_t)sbase)) seterr(GZ_E_TRUNC, at + 32u);
                    else {
                        act = A_STORED;
                        x0 = (uint32_t)(sbase + (at >> 3) + 4 - ma);  // data start, member-relative
                        x1 = w & 0xFFFFu;
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
                    if (hlit > 286 || hdist > 30) seterr(GZ_E_CODES, fill - (uint32_t)bc);
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
                    if (!err && left != 0) seterr(GZ_E_CODES, fill - (uint32_t)bc);  // over-subscribed or incomplete (or empty)
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
                                if (i == 0) { seterr(GZ_E_CODES, fill - (uint32_t)bc); break; }
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
                            if (i + rep > total) { seterr(GZ_E_CODES, fill - (uint32_t)bc); break; }
                            while (rep--) s_len[i++] = v;
                        }
                        if (!err && s_len[256] == 0) seterr(GZ_E_CODES, fill - (uint32_t)bc);  // missing end-of-block code
                    }
                    if (!err) {
                        act = A_BUILD;
                        x0 = (uint32_t)hlit;
                        x1 = (uint32_t)hdist;
                    }
                } else {
                    seterr(GZ_E_BTYPE, fill - (uint32_t)bc);
                }
                nbp = fill - (uint32_t)bc;
                const int64_t lim = 8 * ((int64_t)mz - 8 - (int64_t)sbase);
                if ((int64_t)(err ? err_bits : nbp) > lim) {  // the header ran out of input first
                    err = GZ_E_TRUNC;
                    act = A_ERR;
                }
            }
            act = bfl(act);
            x0 = bfl(x0);
            x1 = bfl(x1);
            final_seen = bfl(fin) != 0;
            GZ_STAMP(1);
            GZ_COUNT(1);
            if (act == A_ERR) break;
            if (act == A_STORED) {
                const uint32_t start = x0, len = x1;
                int32_t e2 = GZ_OK;
                if ((uint64_t)start + len + 8 > mlen) e2 = GZ_E_TRUNC;
                else if (produced + len > cap) e2 = GZ_E_OVER;
                if (CH && e2 == GZ_E_OVER && cut_prod > 0) {
                    soft = true;
                    break;
                }
                if (e2 != GZ_OK) {
                    if (lane == 0) err = e2;
                    break;
                }
                for (uint32_t i = (uint32_t)lane; i < len; i += 64) dst[produced + i] = in[ma + start + i];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                produced += len;
                restage(ma + start + len, 0);
                continue;
            }
            // ---- A_BUILD: canonical codes by ballots, primary tables filled from registers ----
            bp = bfl(nbp);
            const int nl = (int)x0, nd = (int)(x1 & 0xFFFFu);
            const bool fixed = (x1 >> 16) & 1u;
            for (int i = lane; i < (1 << LB); i += 64) s_lit[i] = 0;
            for (int i = lane; i < (1 << DB); i += 64) s_dst[i] = 0;
            __syncthreads();
            const uint64_t below = (1ull << lane) - 1ull;
            bool bad_codes = false;  // wave-uniform (from ballots): loop exits must not depend on lane state
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int base = t ? nl : 0, cntn = t ? nd : nl, bits = t ? DB : LB;
                uint32_t *tab = t ? s_dst : s_lit;
                uint32_t *sent = s_sent + (t ? 288 : 0);
                uint32_t *lim = t ? limD : limL, *lbase = t ? baseD : baseL;
                uint32_t lj[5];
#pragma unroll
                for (int j = 0; j < 5; ++j) lj[j] = 64 * j + lane < cntn ? s_len[base + 64 * j + lane] : 0u;
                uint32_t count[16];
                count[0] = 0;
                int left = 1, mx = 0;
                for (int l = 1; l < 16; ++l) {
                    uint32_t c = 0;
#pragma unroll
                    for (int j = 0; j < 5; ++j) c += (uint32_t)__popcll(__ballot(lj[j] == (uint32_t)l));
                    count[l] = c;
                    left = (left << 1) - (int)c;
                    if (left < 0) break;
                    if (c) mx = l;
                }
                // over-subscribed; incomplete unless a single 1-bit code (zlib's inflate_table)
                if (!fixed && (left < 0 || (mx > 0 && left > 0 && mx != 1))) {
                    bad_codes = true;
                    break;
                }
                uint32_t code = 0, off = 0;
                for (int l = 1; l < 16; ++l) {
                    code = (code + count[l - 1]) << 1;  // first code of length l
                    if (l > 10) {
                        lim[l - 11] = (code + count[l]) << (15 - l);
                        lbase[l - 11] = off - code;
                    }
                    uint32_t run = 0;
#pragma unroll
                    for (int j = 0; j < 5; ++j) {
                        const uint64_t b = __ballot(lj[j] == (uint32_t)l);
                        if (lj[j] == (uint32_t)l) {
                            const uint32_t rank = run + (uint32_t)__popcll(b & below);
                            const int s = 64 * j + lane;
                            const uint32_t e = sym_entry(t, s, l);
                            sent[off + rank] = e;
                            const uint32_t r = __builtin_bitreverse32(code + rank) >> (32 - l);
                            if (l <= bits) {
                                if (e)
                                    for (uint32_t i = r; i < (1u << bits); i += 1u << l) tab[i] = e;
                            } else {
                                tab[r & ((1u << bits) - 1u)] = K_SLOW << 4;
                            }
                        }
                        run += (uint32_t)__popcll(b);
                    }
                    off += count[l];
                }
            }
            if (bad_codes) {
                if (lane == 0) err = GZ_E_CODES;
                break;
            }
            __syncthreads();
            in_block = true;
            if (CH && resume) {  // the tables are built: continue at the chunk's start inside the block
                restage(start_bit >> 3, (uint32_t)(start_bit & 7u));
                resume = false;
            }
            GZ_STAMP(2);
            GZ_COUNT(2);
            continue;
        }
        // ---- Huffman tokens: two 64-bit windows of starts per pass ----
        if (bp > 8u * IN_STAGE - 320u) restage(sbase + (bp >> 3), bp & 7u);
        // The token that would start at bit `pos`: packed length | stop << 6 | kind << 7 |
        // output bytes << 9.  An invalid code is kind K_BAD with, as its length, the bits
        // zlib reads before rejecting it (all 15 of a missing code, the code's own for an
        // undefined symbol), so running out of input first is reported first, as zlib does.
        auto token = [&](uint32_t pos, uint32_t &dist, uint32_t &val) -> uint32_t {
            const uint32_t a = pos >> 5, sh = pos & 31u;
            const uint32_t w0 = s_in32[a], w1 = s_in32[a + 1], w2 = s_in32[a + 2];
            const uint64_t x = (uint64_t)__builtin_amdgcn_alignbit(w1, w0, sh) |
                               (uint64_t)__builtin_amdgcn_alignbit(w2, w1, sh) << 32;
            uint32_t e = s_lit[x & ((1u << LB) - 1u)];
            if (((e >> 4) & 3u) == K_SLOW) e = long_decode(x, limL, baseL, s_sent);
            const uint32_t n1 = e & 15u, eb = (e >> 8) & 15u;
            uint32_t kind = (e >> 4) & 3u;
            uint32_t tl = n1, ol = kind == K_EOB ? 0u : 1u;
            dist = 0;
            val = e >> 16;
            if (!n1 || (kind == K_LEN && eb == X_BADSYM)) {
                tl = n1 ? n1 : 15u;
                kind = K_BAD;
            } else if (kind == K_LEN) {
                val += (uint32_t)(x >> n1) & ((1u << eb) - 1u);
                const uint64_t y = x >> (n1 + eb);
                uint32_t d = s_dst[y & ((1u << DB) - 1u)];
                if (((d >> 4) & 3u) == K_SLOW) d = long_decode(y, limD, baseD, s_sent + 288);
                const uint32_t n2 = d & 15u, db = (d >> 8) & 15u;
                if (!n2 || db == X_BADSYM) {
                    tl = n1 + eb + (n2 ? n2 : 15u);
                    kind = K_BAD;
                } else {
                    dist = (d >> 16) + ((uint32_t)(y >> n2) & ((1u << db) - 1u));
                    tl = n1 + eb + n2 + db;
                    ol = val;
                }
            }
            if (kind == K_BAD) ol = 0;
            const uint32_t stopbit = (kind == K_BAD || kind == K_EOB) ? 64u : 0u;  // the chain ends here
            return tl | stopbit | kind << 7 | ol << 9;
        };
        uint32_t dist0, val0, dist1, val1;
        const uint32_t pk0 = token(bp + (uint32_t)lane, dist0, val0);
        const uint32_t pk1 = token(bp + 64u + (uint32_t)lane, dist1, val1);
        GZ_STAMP(3);
        // The real chain from bit bp: the scalar unit only follows the token
        // lengths (v_readlane, add, bit set); the batch offsets, match slots and
        // capacity cut are then found lane-parallel.
        uint32_t q = 0;
        uint64_t M0 = 0, M1 = 0;
        bool stopped = false;
        while (q < 64) {
            const uint32_t info = (uint32_t)__builtin_amdgcn_readlane((int)pk0, (int)q);
            M0 |= 1ull << q;
            q += info & 63u;
            if (info & 64u) { stopped = true; break; }
        }
        if (!stopped)
            while (q < 128) {
                const uint32_t info = (uint32_t)__builtin_amdgcn_readlane((int)pk1, (int)(q - 64));
                M1 |= 1ull << (q - 64);
                q += info & 63u;
                if (info & 64u) { stopped = true; break; }
            }
        GZ_STAMP(7);
        uint32_t stop = 0;  // 0 window done, 1 end of block, 2 batch full, 3 invalid code
        if (stopped) {
            const uint32_t last = M1 ? 127u - (uint32_t)__builtin_clzll(M1) : 63u - (uint32_t)__builtin_clzll(M0);
            const uint32_t info = last < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)pk0, (int)last)
                                            : (uint32_t)__builtin_amdgcn_readlane((int)pk1, (int)(last - 64));
            stop = ((info >> 7) & 3u) == K_BAD ? 3u : 1u;
        }
        const uint64_t below = (1ull << lane) - 1ull;
        const uint32_t kind0 = (pk0 >> 7) & 3u, kind1 = (pk1 >> 7) & 3u;
        uint32_t olen0 = ((M0 >> lane) & 1u) ? pk0 >> 9 : 0u, olen1 = ((M1 >> lane) & 1u) ? pk1 >> 9 : 0u;
        const uint32_t inc0 = wave_incl_sum(olen0);
        const uint32_t tot0 = (uint32_t)__builtin_amdgcn_readlane((int)inc0, 63);
        const uint32_t inc1 = wave_incl_sum(olen1) + tot0;
        const uint64_t mb0 = __ballot(((M0 >> lane) & 1u) && kind0 == K_LEN && olen0);
        const uint64_t mb1 = __ballot(((M1 >> lane) & 1u) && kind1 == K_LEN && olen1);
        const uint32_t mr0 = (uint32_t)__popcll(mb0 & below), mr1 = (uint32_t)__popcll(mb0) + (uint32_t)__popcll(mb1 & below);
        const int opos0 = (int)(nb + inc0 - olen0), opos1 = (int)(nb + inc1 - olen1);
        const int midx0 = (int)(nm + mr0), midx1 = (int)(nm + mr1);
        // batch capacity: the first chain token that does not fit ends this pass before it
        const uint64_t fb0 = __ballot(olen0 && (nb + inc0 > (uint32_t)OBUF || (kind0 == K_LEN && nm + mr0 >= (uint32_t)MLCAP)));
        const uint64_t fb1 = __ballot(olen1 && (nb + inc1 > (uint32_t)OBUF || (kind1 == K_LEN && nm + mr1 >= (uint32_t)MLCAP)));
        uint32_t acc = (uint32_t)__builtin_amdgcn_readlane((int)inc1, 63);
        if (fb0 | fb1) {
            const uint32_t first = fb0 ? (uint32_t)__builtin_ctzll(fb0) : 64u + (uint32_t)__builtin_ctzll(fb1);
            if (first < 64) {
                M0 &= (1ull << first) - 1ull;
                M1 = 0;
                acc = (uint32_t)__builtin_amdgcn_readlane(opos0, (int)first) - nb;
            } else {
                M1 &= (1ull << (first - 64)) - 1ull;
                acc = (uint32_t)__builtin_amdgcn_readlane(opos1, (int)(first - 64)) - nb;
            }
            q = first;
            stop = 2;
            olen0 = ((M0 >> lane) & 1u) ? olen0 : 0u;
            olen1 = ((M1 >> lane) & 1u) ? olen1 : 0u;
        }
        const uint32_t nmat = (uint32_t)__popcll(mb0 & M0) + (uint32_t)__popcll(mb1 & M1);
        const bool on0 = olen0 != 0, on1 = olen1 != 0;  // chain tokens with output (not end of block)
        // The first error in stream order, as zlib meets it: per chain token,
        // its bits running past the deflate data (the trailer's 8 bytes are not
        // input), then a distance too far back, then output past ISIZE; the
        // window-0 tokens precede the window-1 ones; an invalid code ends the
        // chain, so every token before it comes first.
        const int64_t lim = 8 * ((int64_t)mz - 8 - (int64_t)sbase);
        auto tok_bad = [&](uint64_t M, uint32_t pk, uint32_t start, bool on, uint32_t kind, uint32_t dist, int opos,
                           uint32_t olen) -> int32_t {
            const uint32_t tl = pk & 63u;
            if (!((M >> lane) & 1ull)) return GZ_OK;
            if ((int64_t)start + tl > lim) return GZ_E_TRUNC;
            if (on && kind == K_LEN && dist > produced + (uint32_t)opos && from_header) return GZ_E_FAR;
            if (on && produced + (uint32_t)opos + olen > cap) return GZ_E_OVER;
            return GZ_OK;
        };
        const int32_t bad0 = tok_bad(M0, pk0, bp + (uint32_t)lane, on0, kind0, dist0, opos0, olen0);
        const int32_t bad1 = tok_bad(M1, pk1, bp + 64u + (uint32_t)lane, on1, kind1, dist1, opos1, olen1);
        const uint64_t bm0 = __ballot(bad0 != GZ_OK), bm1 = __ballot(bad1 != GZ_OK);
        if (bm0 | bm1) {
            const int32_t b0 = bm0 ? __builtin_amdgcn_readlane(bad0, (int)__builtin_ctzll(bm0))
                                   : __builtin_amdgcn_readlane(bad1, (int)__builtin_ctzll(bm1));
            if (CH && b0 == GZ_E_OVER && cut_prod > 0) {  // the slot is full: the chunk ends at the last cut
                soft = true;
                break;
            }
            if (lane == 0) err = b0;
            break;
        }
        if (stop == 3) {  // an invalid code on the chain
            if (lane == 0) err = GZ_E_CODE;
            break;
        }
        if (stop == 2 && q == 0 && nb == 0) {  // the first token does not fit an empty batch: no progress
            if (lane == 0) err = GZ_E_STALL;
            break;
        }
        if (on0 && kind0 == K_LIT) {
            s_ob[opos0] = (OT)val0;
            s_ref[opos0] = 0;
        } else if (on0 && kind0 == K_LEN) {
            s_mpl[midx0] = (uint32_t)opos0 | val0 << 16;
            s_md[midx0] = (uint16_t)dist0;
        }
        if (on1 && kind1 == K_LIT) {
            s_ob[opos1] = (OT)val1;
            s_ref[opos1] = 0;
        } else if (on1 && kind1 == K_LEN) {
            s_mpl[midx1] = (uint32_t)opos1 | val1 << 16;
            s_md[midx1] = (uint16_t)dist1;
        }
        nb = bfl(nb + acc);  // (readfirstlane: the batch state stays in SGPRs)
        nm = bfl(nm + nmat);
        bp = bfl(bp + q);
        if (sbase + (bp >> 3) > mz) {  // consumed past the member: truncated
            if (lane == 0) err = GZ_E_TRUNC;
            break;
        }
        if (stop == 1) in_block = false;
        GZ_STAMP(1);
        GZ_COUNT(3);
        if (stop == 0 || nb == 0) continue;
        // ---- flush: expand the matches, resolve them, store the batch ----
        __syncthreads();
        for (uint32_t k = (uint32_t)lane; k < nm; k += 64) {
            const uint32_t pl = s_mpl[k], mp = pl & 0xFFFFu, len = pl >> 16;
            const uint16_t d = s_md[k];
            for (uint32_t i = 0; i < len; ++i) s_ref[mp + i] = d;
        }
        __syncthreads();
        GZ_STAMP(4);
        GZ_COUNT(4);
        if (nm) {
            for (;;) {
                bool more = false;
                for (uint32_t b0 = 0; b0 < nb; b0 += 64 * 8) {
                    uint32_t d[8], v[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const uint32_t qq = b0 + (uint32_t)lane + 64u * j;
                        d[j] = qq < nb ? (uint32_t)s_ref[qq] : 0u;
                    }
#pragma unroll
                    for (int j = 0; j < 8; ++j) {  // history sources: all loads in flight
                        const int src = (int)(b0 + (uint32_t)lane + 64u * j) - (int)d[j];
                        const int64_t hp = (int64_t)produced + src;
                        if (CH && hp < 0)  // before the chunk: a window marker (distances are <= 32 KiB)
                            v[j] = d[j] && src < 0 ? 256u + (uint32_t)(32768 + hp) : 0u;
                        else
                            v[j] = d[j] && src < 0 ? (uint32_t)dst[hp] : 0u;
                    }
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        if (!d[j]) continue;
                        const uint32_t qq = b0 + (uint32_t)lane + 64u * j;
                        const int src = (int)qq - (int)d[j];
                        if (src >= 0) {
                            const uint32_t d2 = s_ref[src];
                            if (d2) {  // the source is itself a copy: follow it
                                s_ref[qq] = (uint16_t)(d[j] + d2);
                                more = true;
                                continue;
                            }
                            v[j] = s_ob[src];
                        }
                        s_ob[qq] = (OT)v[j];
                        s_ref[qq] = 0;
                    }
                }
                __syncthreads();
                GZ_COUNT(5);
                if (!__any(more)) break;
            }
        }
        GZ_STAMP(5);
        for (uint32_t qq = (uint32_t)lane; qq < nb; qq += 64) dst[produced + qq] = s_ob[qq];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        __syncthreads();
        produced += nb;
        nb = 0;
        nm = 0;
        if constexpr (CH) {
            cut_bit = 8 * sbase + bp;
            cut_hdr = in_block ? blk_bit : cut_bit;
            cut_prod = produced;
        }
        GZ_STAMP(6);
        GZ_COUNT(6);
    }
    if constexpr (CH) {
        if (lane == 0) {
            const uint64_t at = 8 * sbase + bp;
            // the final block ended here; the host checks that the trailer follows it and the
            // fold reads its CRC from the member's last 8 bytes (no word shared between chunks:
            // a chunk decoding from a wrong header pick may also "see" a final block)
            if (!err && final_seen && !soft && ((at + 7) >> 3) + 8 > mz) err = GZ_E_TRUNC;
            ca.status[c] = err;
            ca.len[c] = soft ? cut_prod : produced;
            ca.end_bit[c] = soft ? cut_bit : at;
            ca.end_hdr[c] = soft ? cut_hdr : at;
            ca.flags[c] = (final_seen && !soft ? (uint32_t)GZC_FINAL : 0u) | (soft ? (uint32_t)GZC_SOFT : 0u);
            ca.next[c] = handed ? tgt : ~0u;
        }
        return;
    }
    // ---- trailer ----
    if (lane == 0) {
        if (!err) {
            const uint64_t t = sbase + ((bp + 7u) >> 3);  // absolute
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
    int32_t s0 = status[m];
    const bool pre = (s0 & GZ_VERIFIED) != 0;  // a chunked member: decoded and CRC-checked already
    s0 &= ~GZ_VERIFIED;
    if (s0 == GZ_OK && !pre) {
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
    if (lane == 0 && pre) status[m] = s0;
    if (lane == 0 && (pre ? s0 : status[m]) != GZ_OK) {
        atomicAdd(&bad[0], 1u);
        atomicMin(&bad[1], (uint32_t)m);
    }
}

// ---- chunked members: block-header search ----------------------------------------
// A block of 4 waves per chunk scans bit offsets from the chunk's nominal start, a
// staged 4 KiB of input at a time.  Every offset of the stage is tested first for
// a dynamic-block header whose fixed fields are legal and whose code-length code is
// complete (Kraft sum exactly 1, as zlib requires) -- about 0.09 % of offsets in
// real DEFLATE data survive -- and the survivors are then checked in full, a wave
// per survivor (wave_header_ok); the lowest passing offset is the chunk's start.  A wrong pick only costs time: a chunk is used only where its
// predecessor's decode hands over to it.
constexpr int FIND_STAGE = 4096;  // staged bytes per step
constexpr int FIND_THREADS = 256;
constexpr int FIND_CAP = 2048;    // survivors checked per stage (more: the rest are passed over)

// The full check of a dynamic-block header at stage bit `at`, by a whole wave
// (at: wave-uniform) -- the code lengths with their repeat rules, an
// end-of-block code, and zlib's inflate_table rules (no over-subscribed code; no
// incomplete lit/len or distance code except a single one-bit code; no distance
// code at all is allowed).  The code-length code's
// canonical table is built by the lanes holding its 19 lengths (ballot counts,
// rank in symbol order) into `tab` (128 entries); then the code-length symbols
// are decoded speculatively -- lane i decodes the symbol that would start at bit
// bp + i, the scalar unit follows the chain from bp -- and each pass takes the
// chain's lengths at once: positions by a prefix sum of the symbols' counts, a
// '16' repeating the last length before it by a last-set scan, Kraft sums and
// nonzero / one-bit counts per code by wave sums, the end-of-block length where
// position 256 falls.  An over-subscribed code fails at the end of its pass.
template <class Peek>
__device__ bool wave_header_ok(const Peek &peek, uint32_t at, int64_t lim, uint16_t *tab) {
    const int lane = lane_id();
    const uint32_t x = peek(at);
    const int hlit = (int)((x >> 3) & 31u) + 257, hdist = (int)((x >> 8) & 31u) + 1,
              hclen = (int)((x >> 13) & 15u) + 4;
    if (hlit > 286 || hdist > 30) return false;
    uint32_t sym = 31, len = 0;
    if (lane < 19) {
        sym = c_cl_order[lane];
        if (lane < hclen) len = peek(at + 17 + 3 * (uint32_t)lane) & 7u;
    }
    uint32_t first = 0, cnt_prev = 0, my_first = 0;
    for (int l = 1; l <= 7; ++l) {
        first = (first + cnt_prev) << 1;  // the first code of length l
        if (len == (uint32_t)l) my_first = first;
        cnt_prev = (uint32_t)__popcll(__ballot(len == (uint32_t)l));
    }
    uint32_t rank = 0;  // among the codes of the same length, in symbol order
    for (int j = 0; j < 19; ++j) {
        const uint32_t lj = (uint32_t)__builtin_amdgcn_readlane((int)len, j);
        const uint32_t sj = (uint32_t)__builtin_amdgcn_readlane((int)sym, j);
        rank += lj == len && sj < sym ? 1u : 0u;
    }
    for (int i = lane; i < 128; i += 64) tab[i] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (len) {
        const uint32_t r = __builtin_bitreverse32(my_first + rank) >> (32 - len);
        for (uint32_t i = r; i < 128; i += 1u << len) tab[i] = (uint16_t)(len | sym << 4);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const uint32_t total = (uint32_t)(hlit + hdist);
    uint32_t bp = at + 17 + 3 * (uint32_t)hclen;  // wave-uniform from here on
    uint32_t got = 0, prev = 0;                   // lengths so far; the last one (bit 8: there is one)
    uint32_t krl = 0, krd = 0, nzl = 0, nzd = 0, n1l = 0, n1d = 0;
    bool eob = false;
    auto wsum = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum(v), 63); };
    while (got < total) {
        const uint32_t w = peek(bp + (uint32_t)lane);
        const uint32_t e = tab[w & 127u];
        const uint32_t l = e & 15u, s = e >> 4;
        const uint32_t xb = s == 16 ? 2u : s == 17 ? 3u : s == 18 ? 7u : 0u;
        const uint32_t tl = l ? l + xb : 0u;
        const uint32_t xv = (w >> l) & ((1u << xb) - 1u);
        const uint32_t n = s < 16 ? 1u : s == 18 ? 11u + xv : 3u + xv;
        uint64_t M = 0;  // the real chain from bp
        bool broken = false;
        for (uint32_t q = 0; q < 64;) {
            M |= 1ull << q;
            const uint32_t t = (uint32_t)__builtin_amdgcn_readlane((int)tl, (int)q);
            if (t == 0) { broken = true; break; }  // (no code: impossible for a complete code)
            q += t;
        }
        if (broken) return false;
        const bool real = (M >> lane) & 1ull;
        const uint32_t nn = real ? n : 0u;
        const uint32_t P = got + wave_incl_sum(nn) - nn;  // this symbol's first length position
        const bool valid = real && P < total;
        const uint64_t V = __ballot(valid);
        const int lv = 63 - __builtin_clzll(V);           // the pass ends with this symbol
        const uint32_t endP = (uint32_t)__builtin_amdgcn_readlane((int)(P + nn), lv);
        if (endP > total) return false;                   // a repeat past the last length
        uint32_t sc = valid && s != 16 ? 0x100u | (s < 16 ? s : 0u) : 0u;
        DPP_SCAN(sc, last_set);
        const uint32_t ex = wave_prev(sc);
        const uint32_t before = (ex & 0x100u) ? ex : prev;
        if (__ballot(valid && s == 16 && !(before & 0x100u))) return false;  // '16' with no length before it
        const uint32_t v = s < 16 ? s : s == 16 ? (before & 0xFFu) : 0u;
        const uint32_t nl = !valid ? 0u : P >= (uint32_t)hlit ? 0u : ((uint32_t)hlit - P < nn ? (uint32_t)hlit - P : nn);
        const uint32_t nd = valid ? nn - nl : 0u;
        const uint32_t wg = v ? 1u << (15 - v) : 0u;
        krl += wsum(nl * wg);
        krd += wsum(nd * wg);
        nzl += wsum(v ? nl : 0u);
        nzd += wsum(v ? nd : 0u);
        n1l += wsum(v == 1 ? nl : 0u);
        n1d += wsum(v == 1 ? nd : 0u);
        eob = eob || __ballot(valid && P <= 256u && 256u < P + nn && v != 0) != 0;
        if (krl > 32768u || krd > 32768u) return false;
        got = endP;
        prev = 0x100u | (uint32_t)__builtin_amdgcn_readlane((int)v, lv);
        bp += (uint32_t)lv + (uint32_t)__builtin_amdgcn_readlane((int)tl, lv);
    }
    if (!eob) return false;
    if (krl != 32768u && !(nzl == 1 && n1l == 1)) return false;
    if (krd != 32768u && !(nzd == 0 || (nzd == 1 && n1d == 1))) return false;
    return (int64_t)bp <= lim;
}

__global__ __launch_bounds__(FIND_THREADS) void k_gz_find(const uint8_t *__restrict__ in, uint64_t ma, uint64_t mz,
                                                         const uint64_t *__restrict__ nominal, uint64_t span,
                                                         uint64_t *__restrict__ found, uint32_t *__restrict__ stats) {
    __shared__ __attribute__((aligned(16))) uint32_t s_in32[FIND_STAGE / 4 + 4];
    __shared__ uint32_t s_surv[FIND_CAP];
    __shared__ uint16_t s_tab[FIND_THREADS / 64][128];
    __shared__ uint32_t s_n;
    __shared__ unsigned long long s_best;
    const int tid = (int)threadIdx.x, lane = tid & 63;
    const uint64_t c = blockIdx.x;
    const uint64_t q0 = nominal[c];
    const uint64_t lim = 8 * (mz - 8);  // the deflate data ends before the trailer
    uint64_t res = GZ_NO_BIT;
    const uint64_t qz = q0 + span < lim ? q0 + span : lim;
    uint32_t n_stages = 0, n_checks = 0;  // (stats: diagnostic)
    unsigned long long cyc_scan = 0, cyc_check = 0;
    for (uint64_t base = q0; base < qz && res == GZ_NO_BIT;) {
        const uint64_t sb = (base >> 3) & ~(uint64_t)15;  // staged from this byte
        for (int k = tid; k < FIND_STAGE / 16; k += FIND_THREADS) {
            const uint64_t q = sb + 16 * (uint64_t)k;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (q + 16 <= mz) v = *reinterpret_cast<const uint4 *>(in + q);
            else if (q < mz) {
                uint32_t w[4] = {0, 0, 0, 0};
                for (int b = 0; b < 16 && q + b < mz; ++b) w[b >> 2] |= (uint32_t)in[q + b] << (8 * (b & 3));
                v = make_uint4(w[0], w[1], w[2], w[3]);
            }
            reinterpret_cast<uint4 *>(s_in32)[k] = v;
        }
        if (tid == 0) {
            reinterpret_cast<uint4 *>(s_in32)[FIND_STAGE / 16] = make_uint4(0, 0, 0, 0);
            s_best = GZ_NO_BIT;
            s_n = 0;
        }
        __syncthreads();
        const unsigned long long t0 = stats ? __builtin_amdgcn_s_memtime() : 0ull;
        auto peek = [&](uint32_t pos) -> uint32_t {  // 32 stage bits from bit pos
            const uint32_t a = pos >> 5;
            return __builtin_amdgcn_alignbit(s_in32[a + 1], s_in32[a], pos & 31u);
        };
        // offsets tested from this stage: a full header (<= ~600 B) must fit behind them
        const uint32_t p0 = (uint32_t)(base - 8 * sb);
        const uint32_t pz = 8u * (FIND_STAGE - HDR_ROOM);
        for (uint32_t pb = p0; pb < pz; pb += FIND_THREADS) {
            const uint32_t pos = pb + (uint32_t)tid;
            const uint32_t lo = peek(pos), mid = peek(pos + 32), hi = peek(pos + 64);
            bool ok = 8 * sb + pos < qz && ((lo >> 1) & 3u) == 2u && ((lo >> 3) & 31u) <= 29u &&
                      ((lo >> 8) & 31u) <= 29u;
            if (ok) {
                const int hclen = (int)((lo >> 13) & 15u) + 4;
                const uint64_t y = (((uint64_t)mid << 32 | lo) >> 17) | ((uint64_t)hi << 47);
                uint32_t kraft = 0;
                for (int i = 0; i < hclen; ++i) {
                    const uint32_t l = (uint32_t)(y >> (3 * i)) & 7u;
                    kraft += l ? 1u << (7 - l) : 0u;
                }
                ok = kraft == 128u;
            }
            const uint64_t m = __ballot(ok);
            if (m) {
                uint32_t at = 0;
                if (lane == 0) at = atomicAdd(&s_n, (uint32_t)__popcll(m));
                at = (uint32_t)__shfl(at, 0, 64) + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                if (ok && at < (uint32_t)FIND_CAP) s_surv[at] = pos;
            }
        }
        __syncthreads();
        const unsigned long long t1 = stats ? __builtin_amdgcn_s_memtime() : 0ull;
        const uint32_t n = s_n < (uint32_t)FIND_CAP ? s_n : (uint32_t)FIND_CAP;
        const int wv = tid >> 6;
        for (uint32_t j = (uint32_t)wv; j < n; j += FIND_THREADS / 64) {  // a wave per survivor
            const uint32_t pos = s_surv[j];
            if ((unsigned long long)(8 * sb + pos) >= *(volatile unsigned long long *)&s_best) continue;
            if (wave_header_ok(peek, pos, (int64_t)(lim - 8 * sb), s_tab[wv]) && lane == 0)
                atomicMin(&s_best, (unsigned long long)(8 * sb + pos));
        }
        n_checks += n;
        ++n_stages;
        __syncthreads();
        if (stats) {
            const unsigned long long t2 = __builtin_amdgcn_s_memtime();
            cyc_scan += t1 - t0;
            cyc_check += t2 - t1;
        }
        res = s_best;
        base = 8 * sb + pz;  // the next stage starts where this one's offsets stopped
        __syncthreads();
    }
    if (tid == 0) {
        found[c] = res;
        if (stats) {
            stats[3 * c] = n_stages;
            stats[3 * c + 1] = n_checks;
            stats[3 * c + 2] = (uint32_t)(cyc_check >> 10);  // (kilo-ticks; the scan's in the high half below)
            stats[3 * c + 1] = n_checks | (uint32_t)((cyc_scan >> 10) << 12);
        }
    }
}

// ---- chunked members: the window chain, in stream order ---------------------------
// window[j] = the last 32 KiB of the output through ordered chunk j.  As a map over
// window[j - 1], position i of it is a byte (< 256) or 256 + w (byte w of window
// [j - 1]): the chunk's own slot values, or -- a chunk shorter than the window --
// the tail of window[j - 1].  Maps compose (M_b after M_a: M_b's markers look up
// M_a), so the chain runs in two levels instead of one step per chunk: groups of
// G chunks compose their maps in parallel (A), one block walks the group maps
// (B), and every group applies its chunks' maps from its start window (C).
constexpr int WIN32K = 32768;
constexpr int GZW_THREADS = 1024;
constexpr int GZW_PER = WIN32K / GZW_THREADS;
struct WinMaps {  // ordered chunk j's map, loaded GZW_PER values per thread
    const uint16_t *slots;
    uint32_t cap;
    const uint32_t *order, *len;
    __device__ void load(uint64_t j, int t, uint32_t (&v)[GZW_PER]) const {
        const uint32_t c = order[j], L = len[c];
        const uint16_t *sl = slots + (uint64_t)c * cap;
#pragma unroll
        for (int k = 0; k < GZW_PER; ++k) {
            const int i = t + GZW_THREADS * k;
            const int64_t q = (int64_t)L - WIN32K + i;  // position in the chunk; below 0: window[j - 1]
            v[k] = q >= 0 ? (uint32_t)sl[q] : 256u + (uint32_t)(i + (int)L);
        }
    }
};

// (A) group g's composed map: M_{last} after ... after M_{first}
__global__ __launch_bounds__(GZW_THREADS) void k_gz_wcompose(WinMaps M, uint64_t n, uint64_t G,
                                                            uint16_t *__restrict__ Q) {
    __shared__ uint16_t q[WIN32K];
    const int t = (int)threadIdx.x;
    const uint64_t j0 = (uint64_t)blockIdx.x * G, j1 = j0 + G < n ? j0 + G : n;
    uint32_t nv[GZW_PER];
    M.load(j0, t, nv);
#pragma unroll
    for (int k = 0; k < GZW_PER; ++k) q[t + GZW_THREADS * k] = (uint16_t)nv[k];
    if (j0 + 1 < j1) M.load(j0 + 1, t, nv);
    __syncthreads();
    for (uint64_t j = j0 + 1; j < j1; ++j) {
        uint32_t r[GZW_PER];
#pragma unroll
        for (int k = 0; k < GZW_PER; ++k) r[k] = nv[k] < 256u ? nv[k] : (uint32_t)q[nv[k] - 256u];
        if (j + 1 < j1) M.load(j + 1, t, nv);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < GZW_PER; ++k) q[t + GZW_THREADS * k] = (uint16_t)r[k];
        __syncthreads();
    }
    uint16_t *dst = Q + (uint64_t)blockIdx.x * WIN32K;
#pragma unroll
    for (int k = 0; k < GZW_PER; ++k) dst[t + GZW_THREADS * k] = q[t + GZW_THREADS * k];
}

// (B) the window after every group, in order
__global__ __launch_bounds__(GZW_THREADS) void k_gz_wchain(const uint16_t *__restrict__ Q, uint64_t ng,
                                                          uint8_t *__restrict__ wend) {
    __shared__ uint8_t w[WIN32K];
    const int t = (int)threadIdx.x;
    for (int i = t; i < WIN32K; i += GZW_THREADS) w[i] = 0;
    uint32_t nv[GZW_PER];
    auto load = [&](uint64_t g) {
#pragma unroll
        for (int k = 0; k < GZW_PER; ++k) nv[k] = Q[g * WIN32K + t + GZW_THREADS * k];
    };
    load(0);
    __syncthreads();
    for (uint64_t g = 0; g < ng; ++g) {
        uint32_t r[GZW_PER];
#pragma unroll
        for (int k = 0; k < GZW_PER; ++k) r[k] = nv[k] < 256u ? nv[k] : (uint32_t)w[nv[k] - 256u];
        if (g + 1 < ng) load(g + 1);
        __syncthreads();
        uint8_t *dst = wend + g * WIN32K;
#pragma unroll
        for (int k = 0; k < GZW_PER; ++k) {
            w[t + GZW_THREADS * k] = (uint8_t)r[k];
            dst[t + GZW_THREADS * k] = (uint8_t)r[k];
        }
        __syncthreads();
    }
}

// (C) every chunk's window, groups in parallel from their start windows
__global__ __launch_bounds__(GZW_THREADS) void k_gz_wapply(WinMaps M, uint64_t n, uint64_t G,
                                                          const uint8_t *__restrict__ wend,
                                                          uint8_t *__restrict__ windows) {
    __shared__ uint8_t w[WIN32K];
    const int t = (int)threadIdx.x;
    const uint64_t g = blockIdx.x, j0 = g * G, j1 = j0 + G < n ? j0 + G : n;
    for (int i = t; i < WIN32K; i += GZW_THREADS) w[i] = g ? wend[(g - 1) * WIN32K + i] : (uint8_t)0;
    uint32_t nv[GZW_PER];
    M.load(j0, t, nv);
    __syncthreads();
    for (uint64_t j = j0; j < j1; ++j) {
        uint32_t r[GZW_PER];
#pragma unroll
        for (int k = 0; k < GZW_PER; ++k) r[k] = nv[k] < 256u ? nv[k] : (uint32_t)w[nv[k] - 256u];
        if (j + 1 < j1) M.load(j + 1, t, nv);
        __syncthreads();
        uint8_t *dst = windows + j * WIN32K;
#pragma unroll
        for (int k = 0; k < GZW_PER; ++k) {
            w[t + GZW_THREADS * k] = (uint8_t)r[k];
            dst[t + GZW_THREADS * k] = (uint8_t)r[k];
        }
        __syncthreads();
    }
}

// ---- chunked members: bytes, CRC-32 per chunk ----------------------------------------
constexpr int GZR_THREADS = 256;
__global__ __launch_bounds__(GZR_THREADS) void k_gz_resolve(const uint16_t *__restrict__ slots, uint32_t cap,
                                                           const uint32_t *__restrict__ order,
                                                           const uint32_t *__restrict__ len,
                                                           const uint64_t *__restrict__ pos,
                                                           const uint8_t *__restrict__ windows, uint8_t *__restrict__ out,
                                                           uint32_t *__restrict__ crc, uint32_t *__restrict__ shift,
                                                           X2N x2n, int32_t *__restrict__ status) {
    __shared__ uint32_t T[256];
    __shared__ uint32_t s_p[GZR_THREADS];
    const uint64_t j = blockIdx.x;
    const int t = (int)threadIdx.x;
    for (int i = t; i < 256; i += GZR_THREADS) {
        uint32_t c = (uint32_t)i;
        for (int k = 0; k < 8; ++k) c = c & 1u ? (c >> 1) ^ POLY : c >> 1;
        T[i] = c;
    }
    const uint32_t c = order[j], L = len[c];
    const uint64_t P = pos[j];
    const uint16_t *sl = slots + (uint64_t)c * cap;
    const uint8_t *win = j ? windows + (j - 1) * (uint64_t)WIN32K : windows;
    // a marker w is the byte P - 32768 + w of the stream: before the stream is too far back
    const uint32_t wmin = P >= (uint64_t)WIN32K ? 0u : (uint32_t)(WIN32K - P);
    uint8_t *dst = out + P;
    bool far = false;
    for (uint32_t i0 = 0; i0 < L; i0 += 8 * GZR_THREADS) {  // eight values in flight per thread
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t i = i0 + (uint32_t)t + GZR_THREADS * k;
            v[k] = i < L ? (uint32_t)sl[i] : 0u;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (v[k] >= 256u) {
                far |= v[k] - 256u < wmin || j == 0;
                v[k] = win[v[k] - 256u];
            }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t i = i0 + (uint32_t)t + GZR_THREADS * k;
            if (i < L) dst[i] = (uint8_t)v[k];
        }
    }
    if (__syncthreads_or(far) && t == 0) status[0] = GZ_E_FAR;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // CRC-32 of GZR_THREADS segments, folded with crc32_combine's shift
    const uint32_t seg = ((L + GZR_THREADS - 1u) / GZR_THREADS + 15u) & ~15u;
    const uint32_t la = (uint32_t)t * seg < L ? (uint32_t)t * seg : L;
    const uint32_t lz = la + seg < L ? la + seg : L;
    uint32_t cc = ~0u;
    uint32_t i = la;
    for (; i + 16 <= lz; i += 16) {  // sixteen loads in flight, then the table steps
        uint32_t b[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) b[k] = dst[i + k];
#pragma unroll
        for (int k = 0; k < 16; ++k) cc = T[(cc ^ b[k]) & 255u] ^ (cc >> 8);
    }
    for (; i < lz; ++i) cc = T[(cc ^ dst[i]) & 255u] ^ (cc >> 8);
    s_p[t] = ~cc;
    __syncthreads();
    if (t == 0) {
        const uint32_t xs = x2nmodp(seg, 3, x2n);
        uint32_t tot = L ? s_p[0] : 0u;
        for (int l = 1; l < GZR_THREADS; ++l) {
            const uint32_t sa = (uint32_t)l * seg;
            if (sa >= L) break;
            const uint32_t sln = sa + seg <= L ? seg : L - sa;
            tot = multmodp(sln == seg ? xs : x2nmodp(sln, 3, x2n), tot) ^ s_p[l];
        }
        crc[j] = tot;
        shift[j] = x2nmodp(L, 3, x2n);
    }
}

// the member's CRC-32: crc(A B) = crc(A) x^(8|B|) mod P ^ crc(B).  Pairs (crc,
// x^(8 len)) combine associatively -- (A then B) = (crc_A x_B ^ crc_B, x_A x_B) --
// so the chunks fold as a block reduction in stream order.
// (the member's status gets GZ_VERIFIED: k_inflate skips it, k_gz_crc only counts it)
constexpr int GZF_THREADS = 256;
__global__ __launch_bounds__(GZF_THREADS) void k_gz_crc_fold(const uint32_t *__restrict__ crc,
                                                            const uint32_t *__restrict__ shift, uint64_t n,
                                                            const uint8_t *__restrict__ trailer,
                                                            const int32_t *__restrict__ status,
                                                            int32_t *__restrict__ mstatus) {
    __shared__ uint32_t s_c[GZF_THREADS], s_x[GZF_THREADS];
    const int t = (int)threadIdx.x;
    const uint64_t per = (n + GZF_THREADS - 1) / GZF_THREADS;
    uint32_t c = 0, x = 1u << 31;  // the empty string: crc 0, x^0
    for (uint64_t j = (uint64_t)t * per; j < n && j < (uint64_t)(t + 1) * per; ++j) {
        c = multmodp(shift[j], c) ^ crc[j];
        x = multmodp(x, shift[j]);
    }
    s_c[t] = c;
    s_x[t] = x;
    __syncthreads();
    for (int d = 1; d < GZF_THREADS; d <<= 1) {  // pairs (t, t + d) with t a multiple of 2d
        if ((t & (2 * d - 1)) == 0 && t + d < GZF_THREADS) {
            s_c[t] = multmodp(s_x[t + d], s_c[t]) ^ s_c[t + d];
            s_x[t] = multmodp(s_x[t], s_x[t + d]);
        }
        __syncthreads();
    }
    if (t == 0) {
        int32_t st = status[0];
        const uint32_t want = (uint32_t)trailer[0] | (uint32_t)trailer[1] << 8 | (uint32_t)trailer[2] << 16 |
                              (uint32_t)trailer[3] << 24;
        if (st == GZ_OK && s_c[0] != want) st = GZ_E_CRC;
        mstatus[0] = st | GZ_VERIFIED;
    }
}

hipError_t launch_gz_find(const uint8_t *in, uint64_t ma, uint64_t mz, const uint64_t *nominal, uint64_t n_chunks,
                          uint64_t span, uint64_t *found, uint32_t *stats, hipStream_t st) {
    if (!n_chunks) return hipSuccess;
    hipLaunchKernelGGL(k_gz_find, dim3((unsigned)n_chunks), dim3(FIND_THREADS), 0, st, in, ma, mz, nominal, span,
                       found, stats);
    return hipGetLastError();
}

hipError_t launch_inflate_chunks(const uint8_t *in, const GzChunkArgs &a, uint64_t n_list, hipStream_t st) {
    if (!n_list) return hipSuccess;
    hipLaunchKernelGGL(k_inflate_t<true>, dim3((unsigned)n_list), dim3(64), 0, st, in, (const uint64_t *)nullptr,
                       (uint64_t)0, (const uint32_t *)nullptr, (uint8_t *)nullptr, (int32_t *)nullptr,
                       (uint32_t *)nullptr, a);
    return hipGetLastError();
}

hipError_t launch_gz_windows(const uint16_t *slots, uint32_t cap, const uint32_t *order, const uint32_t *len,
                             uint64_t n_order, uint8_t *windows, uint16_t *gmaps, uint8_t *gwin, hipStream_t st) {
    if (!n_order) return hipSuccess;
    const uint64_t G = gz_window_group(n_order), ng = (n_order + G - 1) / G;
    const WinMaps M{slots, cap, order, len};
    hipLaunchKernelGGL(k_gz_wcompose, dim3((unsigned)ng), dim3(GZW_THREADS), 0, st, M, n_order, G, gmaps);
    hipLaunchKernelGGL(k_gz_wchain, dim3(1), dim3(GZW_THREADS), 0, st, gmaps, ng, gwin);
    hipLaunchKernelGGL(k_gz_wapply, dim3((unsigned)ng), dim3(GZW_THREADS), 0, st, M, n_order, G, gwin, windows);
    return hipGetLastError();
}

hipError_t launch_gz_resolve(const uint16_t *slots, uint32_t cap, const uint32_t *order, const uint32_t *len,
                             const uint64_t *pos, uint64_t n_order, const uint8_t *windows, uint8_t *out,
                             uint32_t *crc, uint32_t *shift, const X2N &x2n, int32_t *status, hipStream_t st) {
    if (!n_order) return hipSuccess;
    hipLaunchKernelGGL(k_gz_resolve, dim3((unsigned)n_order), dim3(GZR_THREADS), 0, st, slots, cap, order, len, pos,
                       windows, out, crc, shift, x2n, status);
    return hipGetLastError();
}

hipError_t launch_gz_crc_fold(const uint32_t *crc, const uint32_t *shift, uint64_t n_order, const uint8_t *trailer,
                              const int32_t *status, int32_t *mstatus, hipStream_t st) {
    hipLaunchKernelGGL(k_gz_crc_fold, dim3(1), dim3(GZF_THREADS), 0, st, crc, shift, n_order, trailer, status, mstatus);
    return hipGetLastError();
}

hipError_t launch_gz_size(const uint8_t *in, uint64_t in_len, const uint64_t *moff, uint64_t n, uint32_t *size,
                          int32_t *status, unsigned long long *total, hipStream_t st, const uint64_t *mend) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_gz_size, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, in, in_len, moff, n, size, status,
                       total, mend);
    return hipGetLastError();
}

hipError_t launch_inflate(const uint8_t *in, const uint64_t *moff, uint64_t n, const uint32_t *ooff, uint8_t *out,
                          int32_t *status, uint32_t *tcrc, hipStream_t st, const uint64_t *mend) {
    if (!n) return hipSuccess;
    GzChunkArgs a{};
    a.mend = mend;
    hipLaunchKernelGGL(k_inflate_t<false>, dim3((unsigned)n), dim3(64), 0, st, in, moff, n, ooff, out, status, tcrc, a);
    return hipGetLastError();
}

// ---- where a file's first member may end -----------------------------------------
// async-compression's GzipDecoder (gzip_file_provider.rs:18, 64; no multiple_members) decodes
// a file's first member and stops.  Without decoding, the member's end is only known as a
// candidate: the next offset where a member header could start (or the file's end).  A thread
// per 16 bytes tests every offset; candidates are rare in DEFLATE data (a 3-byte pattern plus
// the flag byte), so the file lookup (binary search) and atomicMin run for few of them.
__global__ void k_gz_next_header(const uint8_t *__restrict__ in, uint64_t in_len, const uint64_t *__restrict__ foff,
                                 uint64_t n, const uint64_t *__restrict__ from, unsigned long long *__restrict__ next) {
    const uint64_t q0 = 16 * ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x);
    if (q0 >= in_len) return;
    for (uint64_t p = q0; p < q0 + 16 && p + 4 <= in_len; ++p) {
        if (in[p] != 0x1f || in[p + 1] != 0x8b || in[p + 2] != 8 || (in[p + 3] & 0xE0u)) continue;
        uint64_t lo = 0, hi = n;  // the file holding p: foff[f] <= p < foff[f + 1]
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (foff[mid + 1] <= p) lo = mid + 1; else hi = mid;
        }
        if (lo < n && p > from[lo]) atomicMin(&next[lo], (unsigned long long)p);
    }
}

hipError_t launch_gz_next_header(const uint8_t *in, uint64_t in_len, const uint64_t *foff, uint64_t n,
                                 const uint64_t *from, unsigned long long *next, hipStream_t st) {
    if (!n || !in_len) return hipSuccess;
    const uint64_t threads = (in_len + 15) / 16;
    hipLaunchKernelGGL(k_gz_next_header, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, in, in_len, foff, n,
                       from, next);
    return hipGetLastError();
}

hipError_t launch_gz_crc(const uint32_t *ooff, const uint8_t *out, uint64_t n, const uint32_t *tcrc, const X2N &x2n,
                         int32_t *status, uint32_t *bad, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_gz_crc, dim3((unsigned)n), dim3(64), 0, st, ooff, out, n, tcrc, x2n, status, bad);
    return hipGetLastError();
}

}  // namespace sdl
