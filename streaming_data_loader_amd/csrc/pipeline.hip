// pipeline.hip -- device-wide scans, token compaction, per-record framing and
// row assembly (+ MLM masking / CLM labels) on gfx950.
//
// Row assembly restates, for every row of an arena in one launch:
//   TokenizerWrapper::encode_mask framing      rust/src/tokenizer/tokenizer_wrapper.rs:107-134
//   GenTokenizer filter + chunks_mut(S)        rust/src/tasks/gen_batcher.rs:69-94
//   BertData::put_data / mask_batch            rust/src/models/bert_data.rs:40-89
//   GptData::put_data                          rust/src/models/gpt_data.rs:29-45
// with the reference's thread_rng replaced by the seeded Philox contract
// (DESIGN.md "RNG contract").  One wave64 owns one row of S positions; lane l
// holds positions l, l+64, l+128, ... so every plane store is one coalesced
// 256-B wave instruction.
#include "common.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "rows_device.hpp"

namespace sdl {

// ---------------------------------------------------------------------------
// Exclusive scan (reduce -> scan of tile sums -> apply), u32.
// ---------------------------------------------------------------------------
constexpr int SCAN_NT = 256;
constexpr int SCAN_PER = 8;
constexpr int SCAN_TILE = SCAN_NT * SCAN_PER;

__global__ __launch_bounds__(SCAN_NT) void k_scan_reduce(const uint32_t *__restrict__ in, int64_t n,
                                                         uint32_t *__restrict__ sums) {
    __shared__ uint32_t scratch[SCAN_NT / 64];
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_PER;
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_PER; ++k)
        if (base + k < n) s += in[base + k];
    uint32_t tot;
    block_excl_sum<SCAN_NT>(s, &tot, scratch);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SCAN_NT) void k_scan_sums(uint32_t *__restrict__ sums, int64_t nb,
                                                       const uint32_t *carry_in) {
    __shared__ uint32_t scratch[SCAN_NT / 64];
    uint32_t carry = carry_in ? *carry_in : 0u;
    for (int64_t t0 = 0; t0 < nb; t0 += SCAN_TILE) {
        const int64_t base = t0 + (int64_t)threadIdx.x * SCAN_PER;
        uint32_t v[SCAN_PER], s = 0;
#pragma unroll
        for (int k = 0; k < SCAN_PER; ++k) {
            v[k] = base + k < nb ? sums[base + k] : 0u;
            s += v[k];
        }
        uint32_t tot;
        uint32_t ex = block_excl_sum<SCAN_NT>(s, &tot, scratch) + carry;
#pragma unroll
        for (int k = 0; k < SCAN_PER; ++k) {
            if (base + k < nb) sums[base + k] = ex;
            ex += v[k];
        }
        carry += tot;
    }
    if (threadIdx.x == 0) sums[nb] = carry;
}

__global__ __launch_bounds__(SCAN_NT) void k_scan_apply(const uint32_t *__restrict__ in, int64_t n,
                                                        const uint32_t *__restrict__ sums, int64_t nb,
                                                        uint32_t *__restrict__ out) {
    __shared__ uint32_t scratch[SCAN_NT / 64];
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_PER;
    uint32_t v[SCAN_PER], s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_PER; ++k) {
        v[k] = base + k < n ? in[base + k] : 0u;
        s += v[k];
    }
    uint32_t tot;
    uint32_t ex = block_excl_sum<SCAN_NT>(s, &tot, scratch) + sums[blockIdx.x];
#pragma unroll
    for (int k = 0; k < SCAN_PER; ++k) {
        if (base + k < n) out[base + k] = ex;
        ex += v[k];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = sums[nb];
}

// n <= SCAN_SMALL: one workgroup, one launch (a per-record push scans a handful
// of chunk and record counts; three dependent launches would cost more than the scan)
constexpr int SCAN_SMALL_NT = 1024, SCAN_SMALL_PER = 8;
constexpr int64_t SCAN_SMALL = (int64_t)SCAN_SMALL_NT * SCAN_SMALL_PER;
__global__ __launch_bounds__(SCAN_SMALL_NT) void k_scan_small(const uint32_t *__restrict__ in, int64_t n,
                                                              uint32_t *__restrict__ out, const uint32_t *carry_in) {
    __shared__ uint32_t scratch[SCAN_SMALL_NT / 64];
    const uint32_t carry = carry_in ? *carry_in : 0u;
    __syncthreads();  // (the carry may be out[0] itself, rewritten below)
    const int64_t base = (int64_t)threadIdx.x * SCAN_SMALL_PER;
    uint32_t v[SCAN_SMALL_PER], s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_SMALL_PER; ++k) {
        v[k] = base + k < n ? in[base + k] : 0u;
        s += v[k];
    }
    uint32_t tot;
    uint32_t ex = block_excl_sum<SCAN_SMALL_NT>(s, &tot, scratch) + carry;
#pragma unroll
    for (int k = 0; k < SCAN_SMALL_PER; ++k) {
        if (base + k < n) out[base + k] = ex;
        ex += v[k];
    }
    if (threadIdx.x == 0) out[n] = carry + tot;
}

int64_t scan_tmp_words(int64_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE + 1; }

hipError_t launch_exclusive_scan(const uint32_t *in, uint32_t *out, int64_t n, uint32_t *tmp, hipStream_t st,
                                 const uint32_t *carry_in) {
    if (n <= 0) return carry_in ? hipSuccess : hipMemsetAsync(out, 0, sizeof(uint32_t), st);
    if (n <= SCAN_SMALL) {
        hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(SCAN_SMALL_NT), 0, st, in, n, out, carry_in);
        return hipGetLastError();
    }
    const int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)nb), dim3(SCAN_NT), 0, st, in, n, tmp);
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(SCAN_NT), 0, st, tmp, nb, carry_in);
    hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)nb), dim3(SCAN_NT), 0, st, in, n, tmp, nb, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Pipelined segments (kernels.hpp SegChunks): rb[k] = first record whose ids
// are not all in chunks < cb[k], i.e. (first r with off[r] >= cb[k] * CHUNK) - 1
// = ranges[3 cb[k] + 2] - 1; rb[0] = 0, rb[K] = R.
__global__ void k_seg_bounds(const uint32_t *__restrict__ ranges, SegChunks sc, int64_t R, uint32_t *__restrict__ rb) {
    const int k = (int)threadIdx.x;
    if (k > sc.K) return;
    uint32_t v;
    if (k == 0) v = 0;
    else if (k == sc.K) v = (uint32_t)R;
    else {
        const uint32_t q = ranges[3 * sc.cb[k] + 2];
        v = q == 0 ? 0u : q - 1u;
        if (v > (uint32_t)R) v = (uint32_t)R;
    }
    rb[k] = v;
}

hipError_t launch_seg_bounds(const uint32_t *ranges, const SegChunks &sc, int64_t R, uint32_t *rb, hipStream_t st) {
    hipLaunchKernelGGL(k_seg_bounds, dim3(1), dim3(64), 0, st, ranges, sc, R, rb);
    return hipGetLastError();
}

// Exclusive scan of in[a, b) into out[a, b] (out[b] = total), carried from
// out[a] when k > 0 (the previous segment wrote its total there); one
// workgroup of 1024 threads, 8 elements per thread per tile.
constexpr int RSCAN_NT = 1024, RSCAN_PER = 8;
__global__ __launch_bounds__(RSCAN_NT) void k_scan_range(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                         const uint32_t *__restrict__ rb, int k) {
    __shared__ uint32_t scratch[RSCAN_NT / 64];
    const int64_t a = rb[k], b = rb[k + 1];
    uint32_t carry = k > 0 ? out[a] : 0u;
    __syncthreads();  // every thread has read out[a] before it is rewritten
    for (int64_t t0 = a; t0 < b; t0 += (int64_t)RSCAN_NT * RSCAN_PER) {
        const int64_t base = t0 + (int64_t)threadIdx.x * RSCAN_PER;
        uint32_t v[RSCAN_PER], sum = 0;
#pragma unroll
        for (int j = 0; j < RSCAN_PER; ++j) {
            v[j] = base + j < b ? in[base + j] : 0u;
            sum += v[j];
        }
        uint32_t tot;
        uint32_t ex = block_excl_sum<RSCAN_NT>(sum, &tot, scratch) + carry;
#pragma unroll
        for (int j = 0; j < RSCAN_PER; ++j) {
            if (base + j < b) out[base + j] = ex;
            ex += v[j];
        }
        carry += tot;
    }
    if (threadIdx.x == 0) out[b] = carry;
}

hipError_t launch_scan_range(const uint32_t *in, uint32_t *out, const uint32_t *rb, int k, hipStream_t st) {
    hipLaunchKernelGGL(k_scan_range, dim3(1), dim3(RSCAN_NT), 0, st, in, out, rb, k);
    return hipGetLastError();
}

// Rows [g_lo, g_end) of a launch; rows >= g_real are the last batch's padding.
struct RowSpan {
    int64_t g_lo, g_real, g_end;
};
__device__ __forceinline__ RowSpan row_span(const SegSel &s, const uint32_t *row_off, int B, int64_t rows_cap) {
    const uint32_t r0 = s.rb[s.k], r1 = s.rb[s.k + 1];
    RowSpan x;
    x.g_lo = row_off[r0];
    x.g_real = row_off[r1];
    x.g_end = x.g_real;
    if (s.last) {
        int64_t Gpad = (x.g_real + B - 1) / B * B;
        if (Gpad > rows_cap) Gpad = rows_cap;
        x.g_end = Gpad > x.g_real ? Gpad : x.g_real;
    }
    return x;
}

// ---------------------------------------------------------------------------
// Per chunk: record ranges touching its window (so the tokenize kernel never
// binary-searches the offsets serially).
// Also (thread 0) the one-segment record bounds rb = {0, R} and a zeroed error word,
// when given: two launches fewer per call.  And, for a small push, its H2D: the grid copies the
// staged blob from mapped pinned memory (cn16 16-B units; the offsets are then read from there
// too) -- no copy in the stream before it.
__global__ __launch_bounds__(256) void k_chunk_ranges(const uint64_t *__restrict__ off, int64_t R, int64_t n_chunks,
                                                      uint32_t *__restrict__ ranges, uint32_t *__restrict__ rb1,
                                                      uint32_t *__restrict__ zero1, const uint4 *__restrict__ csrc,
                                                      uint4 *__restrict__ cdst, int64_t cn16) {
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (int64_t x = c; x < cn16; x += (int64_t)gridDim.x * 256) cdst[x] = csrc[x];
    if (c == 0) {
        if (rb1) {
            rb1[0] = 0u;
            rb1[1] = (uint32_t)R;
        }
        if (zero1) *zero1 = 0u;
    }
    if (c >= n_chunks) return;
    auto lower = [&](int64_t x) {  // first r in [0, R] with off[r] >= x (R+1 if none)
        int64_t lo = 0, hi = R + 1;
        while (lo < hi) {
            const int64_t m = (lo + hi) >> 1;
            if ((int64_t)off[m] < x) lo = m + 1; else hi = m;
        }
        return lo;
    };
    const int64_t c0 = c * CHUNK;
    ranges[3 * c + 0] = (uint32_t)lower(c0 - HALO_L);
    ranges[3 * c + 1] = (uint32_t)lower(c0 - HALO_L + WIN);
    ranges[3 * c + 2] = (uint32_t)lower(c0);
}

hipError_t launch_chunk_ranges(const uint64_t *off, int64_t R, int64_t N, uint32_t *ranges, hipStream_t st,
                               uint32_t *rb1, uint32_t *zero1, const void *copy_src, void *copy_dst, size_t copy_bytes) {
    const int64_t n_chunks = (N + CHUNK - 1) / CHUNK;
    const int64_t cn16 = copy_src ? (int64_t)((copy_bytes + 15) / 16) : 0;
    if (n_chunks == 0 && cn16 == 0) return hipSuccess;
    int64_t blocks = (n_chunks + 255) / 256;
    const int64_t cb = (cn16 + 255) / 256;
    if (cb > blocks) blocks = cb < 64 ? cb : 64;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_chunk_ranges, dim3((unsigned)blocks), dim3(256), 0, st, off, R, n_chunks, ranges, rb1, zero1,
                       (const uint4 *)copy_src, (uint4 *)copy_dst, cn16);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Per-chunk token lists -> one dense token array in arena order.
// ---------------------------------------------------------------------------
template <int PART>
__global__ __launch_bounds__(256) void k_compact_tokens(const uint32_t *__restrict__ tokc,
                                                        const uint32_t *__restrict__ chunk_cnt,
                                                        const uint32_t *__restrict__ chunk_off, int64_t n_chunks,
                                                        uint32_t *__restrict__ tok, const uint32_t *long_count,
                                                        const uint32_t *__restrict__ chunk_ent,
                                                        const BpeLong *__restrict__ long_list,
                                                        const uint16_t *__restrict__ long_scratch,
                                                        const uint32_t *__restrict__ long_pool, int64_t stride) {
    const int64_t cb = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * COMPACT_CPW;  // the wave's first chunk
    if (cb >= n_chunks) return;
    compact_wave<PART>(cb, tokc, chunk_cnt, chunk_off, n_chunks, tok, long_count, chunk_ent, long_list, long_scratch,
                       long_pool, stride);
}

hipError_t launch_compact_tokens(const uint32_t *tokc, const uint32_t *chunk_cnt, const uint32_t *chunk_off,
                                 int64_t n_chunks, uint32_t *tok, const uint32_t *long_count,
                                 const uint32_t *chunk_ent, const BpeLong *long_list, const uint16_t *long_scratch,
                                 hipStream_t st, const uint32_t *long_pool, int64_t stride) {
    if (n_chunks == 0) return hipSuccess;
    const int64_t waves = (n_chunks + COMPACT_CPW - 1) / COMPACT_CPW;
    // (byte-level BPE / unigram: the long-item copy as its own kernel; one of the two has work)
    hipLaunchKernelGGL(k_compact_tokens<1>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, tokc, chunk_cnt,
                       chunk_off, n_chunks, tok, long_count, chunk_ent, long_list, long_scratch, long_pool, stride);
    if (long_count)
        hipLaunchKernelGGL(k_compact_tokens<2>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, tokc, chunk_cnt,
                           chunk_off, n_chunks, tok, long_count, chunk_ent, long_list, long_scratch, long_pool, stride);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_records(RowParams P, const uint64_t *__restrict__ off, int64_t R, int64_t N,
                                                 const uint32_t *__restrict__ chunk_off, int64_t n_chunks,
                                                 const uint32_t *__restrict__ rec_local, uint32_t *__restrict__ rec_tok,
                                                 uint32_t *__restrict__ rec_cnt, uint32_t *__restrict__ rec_rows,
                                                 SegSel sel) {
    const int64_t r_lo = sel.rb[sel.k], r_hi = sel.rb[sel.k + 1];
    for (int64_t r = r_lo + (int64_t)blockIdx.x * 256 + threadIdx.x; r < r_hi; r += (int64_t)gridDim.x * 256)
        record_one(P, off, r, N, chunk_off, n_chunks, rec_local, rec_tok, rec_cnt, rec_rows);
}

hipError_t launch_records(const RowParams &P, const uint64_t *off, int64_t R, int64_t N, const uint32_t *chunk_off,
                          int64_t n_chunks, const uint32_t *rec_local, uint32_t *rec_tok, uint32_t *rec_cnt,
                          uint32_t *rec_rows, SegSel sel, hipStream_t st) {
    if (R == 0) return hipSuccess;
    const int64_t want = (R + 255) / 256;
    hipLaunchKernelGGL(k_records, dim3((unsigned)(want < 1024 ? want : 1024)), dim3(256), 0, st, P, off, R, N,
                       chunk_off, n_chunks, rec_local, rec_tok, rec_cnt, rec_rows, sel);
    return hipGetLastError();
}

// Row g -> its record (one thread per record writes its rows' entries).
__global__ __launch_bounds__(256) void k_row_map(const uint32_t *__restrict__ row_off, uint32_t *__restrict__ row_rec,
                                                 SegSel sel) {
    const int64_t r_lo = sel.rb[sel.k], r_hi = sel.rb[sel.k + 1];
    for (int64_t r = r_lo + (int64_t)blockIdx.x * 256 + threadIdx.x; r < r_hi; r += (int64_t)gridDim.x * 256)
        for (uint32_t g = row_off[r]; g < row_off[r + 1]; ++g) row_rec[g] = (uint32_t)r;
}

// ---------------------------------------------------------------------------
// Small calls (one segment, <= SMALL_CHUNKS chunks, <= SCAN_SMALL records): the
// chunk scan, compaction, per-record framing, row scan and row map of one
// workgroup in one launch instead of five (a per-record push is bound by
// launches, not by these few thousand ids).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void block_scan_small(const uint32_t *__restrict__ in, int64_t n, uint32_t *__restrict__ out,
                                                 uint32_t *scratch) {
    const int64_t base = (int64_t)threadIdx.x * SCAN_SMALL_PER;
    uint32_t v[SCAN_SMALL_PER], s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_SMALL_PER; ++k) {
        v[k] = base + k < n ? in[base + k] : 0u;
        s += v[k];
    }
    uint32_t tot;
    uint32_t ex = block_excl_sum<SCAN_SMALL_NT>(s, &tot, scratch);
#pragma unroll
    for (int k = 0; k < SCAN_SMALL_PER; ++k) {
        if (base + k < n) out[base + k] = ex;
        ex += v[k];
    }
    if (threadIdx.x == 0) out[n] = tot;
}

hipError_t launch_row_map(const uint32_t *row_off, int64_t R, uint32_t *row_rec, SegSel sel, hipStream_t st) {
    if (R == 0) return hipSuccess;
    const int64_t want = (R + 255) / 256;
    hipLaunchKernelGGL(k_row_map, dim3((unsigned)(want < 1024 ? want : 1024)), dim3(256), 0, st, row_off, row_rec, sel);
    return hipGetLastError();
}

// occupancy asked of the compiler (r03i): MR <= 2 Philox rows at 7 waves per SIMD
// (k_rows<2>: 74 -> 71 VGPRs, no spills; mlm rows 0.270 -> 0.262 ms, multi-label
// 0.080 -> 0.074; 8 spills and is slower); MR >= 4 and rng_mode 1 as they come
// (asking 5-6 of them spills)
constexpr int ROWS_WAVES = 7;
constexpr int ROWS_WAVES4 = 1;
constexpr int ROWS_WAVES_RM1 = 6;  // (r04: left to the compiler, 103 VGPRs, 4 waves: rows 0.347 ms; 7 spills 20 B)
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
#define CC_QR(a, b, c, d)                                                         \
    a += b; d ^= a; d = rotl32(d, 16); c += d; b ^= c; b = rotl32(b, 12);         \
    a += b; d ^= a; d = rotl32(d, 8);  c += d; b ^= c; b = rotl32(b, 7);
// ChaCha12 block `ctr` of key k (stream 0)
__device__ __forceinline__ void chacha12_block(const uint32_t (&k)[8], uint32_t ctr, uint32_t (&o)[16]) {
    uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
    uint32_t x4 = k[0], x5 = k[1], x6 = k[2], x7 = k[3], x8 = k[4], x9 = k[5], x10 = k[6], x11 = k[7];
    uint32_t x12 = ctr, x13 = 0u, x14 = 0u, x15 = 0u;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        CC_QR(x0, x4, x8, x12) CC_QR(x1, x5, x9, x13) CC_QR(x2, x6, x10, x14) CC_QR(x3, x7, x11, x15)
        CC_QR(x0, x5, x10, x15) CC_QR(x1, x6, x11, x12) CC_QR(x2, x7, x8, x13) CC_QR(x3, x4, x9, x14)
    }
    o[0] = x0 + 0x61707865u; o[1] = x1 + 0x3320646eu; o[2] = x2 + 0x79622d32u; o[3] = x3 + 0x6b206574u;
    o[4] = x4 + k[0]; o[5] = x5 + k[1]; o[6] = x6 + k[2]; o[7] = x7 + k[3];
    o[8] = x8 + k[4]; o[9] = x9 + k[5]; o[10] = x10 + k[6]; o[11] = x11 + k[7];
    o[12] = x12 + ctr; o[13] = x13; o[14] = x14; o[15] = x15;
}

// A row's blocks differ only in the counter word x12, so of the first column round only the
// quarter round through x12 changes from block to block: ChaRow holds the other three's results
// (x13 = x14 = x15 = 0: the counter's high word and stream 0), computed once per row.
struct ChaRow {
    uint32_t k[8];
    uint32_t c[12];  // (x1, x5, x9, x13), (x2, x6, x10, x14), (x3, x7, x11, x15) after round 1's column QRs
};
__device__ __forceinline__ void chacha_row_init(ChaRow &R, const uint32_t (&k)[8]) {
#pragma unroll
    for (int q = 0; q < 8; ++q) R.k[q] = k[q];
    uint32_t x1 = 0x3320646eu, x5 = k[1], x9 = k[5], x13 = 0u;
    uint32_t x2 = 0x79622d32u, x6 = k[2], x10 = k[6], x14 = 0u;
    uint32_t x3 = 0x6b206574u, x7 = k[3], x11 = k[7], x15 = 0u;
    CC_QR(x1, x5, x9, x13) CC_QR(x2, x6, x10, x14) CC_QR(x3, x7, x11, x15)
    R.c[0] = x1; R.c[1] = x5; R.c[2] = x9; R.c[3] = x13;
    R.c[4] = x2; R.c[5] = x6; R.c[6] = x10; R.c[7] = x14;
    R.c[8] = x3; R.c[9] = x7; R.c[10] = x11; R.c[11] = x15;
}
// = chacha12_block(R.k, ctr, o)
__device__ __forceinline__ void chacha12_block_row(const ChaRow &R, uint32_t ctr, uint32_t (&o)[16]) {
    uint32_t x0 = 0x61707865u, x4 = R.k[0], x8 = R.k[4], x12 = ctr;
    CC_QR(x0, x4, x8, x12)
    uint32_t x1 = R.c[0], x5 = R.c[1], x9 = R.c[2], x13 = R.c[3];
    uint32_t x2 = R.c[4], x6 = R.c[5], x10 = R.c[6], x14 = R.c[7];
    uint32_t x3 = R.c[8], x7 = R.c[9], x11 = R.c[10], x15 = R.c[11];
    CC_QR(x0, x5, x10, x15) CC_QR(x1, x6, x11, x12) CC_QR(x2, x7, x8, x13) CC_QR(x3, x4, x9, x14)
#pragma unroll
    for (int r = 1; r < 6; ++r) {
        CC_QR(x0, x4, x8, x12) CC_QR(x1, x5, x9, x13) CC_QR(x2, x6, x10, x14) CC_QR(x3, x7, x11, x15)
        CC_QR(x0, x5, x10, x15) CC_QR(x1, x6, x11, x12) CC_QR(x2, x7, x8, x13) CC_QR(x3, x4, x9, x14)
    }
    const uint32_t (&k)[8] = R.k;
    o[0] = x0 + 0x61707865u; o[1] = x1 + 0x3320646eu; o[2] = x2 + 0x79622d32u; o[3] = x3 + 0x6b206574u;
    o[4] = x4 + k[0]; o[5] = x5 + k[1]; o[6] = x6 + k[2]; o[7] = x7 + k[3];
    o[8] = x8 + k[4]; o[9] = x9 + k[5]; o[10] = x10 + k[6]; o[11] = x11 + k[7];
    o[12] = x12 + ctr; o[13] = x13; o[14] = x14; o[15] = x15;
}

// rng_mode 1, rows that were not walked beside the tokenizer (rand_pre_slot < 0: chunk >= 1 past
// the byte-length guess, or every row when nothing was): k_rows' LATE pass walks them in place, up
// to 4 rows a wave, 16 lanes a row.  Per window of 16 ChaCha12 blocks the row's 16 lanes each
// compute one block in registers; the row walks the 256 words (rand_walk_lanes' acceptance test),
// each handed to the whole row by DPP row_newbcast, and lane 0 puts each swap straight into next()
// (an LDS atomicMin, as rand_set_bits does from stored indices; a rejected word or a self swap
// targets the dummy slot S); then the row's lanes follow [0, k)'s chains into its mask bits.  The walk is one dependent chain per row (a word's
// test needs the previous word's outcome: lo32(v * n) moves with n like a hash, so guessing n for
// later words and iterating to a fixed point converged lane by lane and measured ~25 us a row);
// these rows are few (~3 % of the bench's), so the chains' latency hides across the waves.
// nx: [4][S + 1], bt: [4][bw] (wave LDS); a lane's group's row is (rec, chunk) when its group <
// nrows.
__device__ __forceinline__ void rand_rows16(const RowParams &P, int nrows, uint64_t rec, uint32_t chunk,
                                            uint32_t *__restrict__ nx,
                                            uint32_t *__restrict__ bt, int bw, int lane) {
    constexpr uint32_t NONE = 0xFFFFFFFFu;
    const int grp = lane >> 4, gl = lane & 15;
    const int S = P.S, kmask = P.mask_length < S ? P.mask_length : S;
    const int i0 = kmask > 1 ? kmask : 1;
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
    const bool active = grp < nrows;
    const uint32_t key[8] = {(uint32_t)P.seed, (uint32_t)(P.seed >> 32), (uint32_t)rec, (uint32_t)(rec >> 32), chunk,
                             0u, 0u, 0u};
    ChaRow cr;
    chacha_row_init(cr, key);
    uint32_t *gnx = nx + (S + 1) * grp, *gbt = bt + bw * grp;
    for (int x = gl; x <= S; x += 16) gnx[x] = NONE;
    for (int x = gl; x < bw; x += 16) gbt[x] = 0u;
    int i = active ? S - 1 : 0;  // (the walk's state: lane 0 of the row's)
    uint32_t n = (uint32_t)i + 1u, zone = (n << __builtin_clz(n)) - 1u;
    for (uint32_t blk = 0;; blk += 16) {
        // wave-uniform: stop when no row of the wave has steps left
        const int irow = __builtin_amdgcn_update_dpp(0, i, 0x150, 0xF, 0xF, false);  // row_newbcast:0
        if (!__any(irow >= i0)) break;
        uint32_t o[16];
        chacha12_block_row(cr, blk + (uint32_t)gl, o);
        // the row's 256 words in order -- block (lane) b's word q by row_newbcast:b, in registers:
        // no LDS round trip on the chain.  Every lane runs the walk; lane 0's is the row's.
        static_for<0, 16>([&](auto bc) {
            constexpr int b = decltype(bc)::value;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const uint32_t x = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)o[q], 0x150 + b, 0xF, 0xF, false);
                const uint64_t m = (uint64_t)x * n;
                const bool acc = i >= i0 && (uint32_t)m <= zone;
                const uint32_t j = (uint32_t)(m >> 32);
                if (gl == 0) atomicMin(&gnx[acc && j != (uint32_t)i ? j : (uint32_t)S], (uint32_t)i);
                i -= acc ? 1 : 0;
                n = (uint32_t)i + 1u;
                zone = (n << __builtin_clz(n)) - 1u;
            }
        });
    }
    wave_sync();
    if (active)
        for (int x = gl; x < kmask; x += 16) {
            uint32_t p = (uint32_t)x;
            for (uint32_t q = gnx[p]; q != NONE; q = gnx[p]) p = q;
            atomicOr(&gbt[p >> 5], 1u << (p & 31));
        }
    wave_sync();
}

// RM1: MLM under rng_mode 1 (the rows' mask words from k_mask_bits_rec, or walked here).  A template flag, not
// a runtime branch: the mask-word registers would cost the Philox path a wave
// per SIMD (k_rows<2>: 80 -> 82 VGPRs, 6 -> 5 waves, 0.267 -> 0.295 ms).
// LATE (RM1 only): the second pass over the rows the first one left (no mask bits from beside the
// tokenizer): its waves walk their masks in place, 4 rows at a time (rand_rows16).
template <int MR, bool RM1, bool LATE = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MR >= 4 ? ROWS_WAVES4 : LATE ? 4 : RM1 ? ROWS_WAVES_RM1 : ROWS_WAVES, 8))) void k_rows(RowParams P, const uint32_t *__restrict__ tok,
                                              const uint32_t *__restrict__ rec_tok, const uint32_t *__restrict__ rec_cnt,
                                              const uint32_t *__restrict__ row_off, const uint32_t *__restrict__ row_rec,
                                              SegSel sel, int64_t rows_cap, RowOut out) {
    const int lane = lane_id();
    const int wid = (int)(threadIdx.x >> 6);
    // (LATE: a wave's LDS for rand_rows16 -- 4 windows, 4 next() arrays + dummy slots, 4 rows' bits)
    constexpr int NXS = 256 * MR + 1, BW = 8 * MR;
    __shared__ __attribute__((aligned(16))) uint32_t s_rw[LATE ? 4 : 1][LATE ? 4 * (NXS + BW) : 1];
    const RowSpan rs = row_span(sel, row_off, P.B, rows_cap);
    const int64_t G = rs.g_real;
    const DirectDst &dd = out.direct;
    const int64_t g_end = dd.cap ? rs.g_real : rs.g_end;  // (direct: the host batch keeps its own padding)
    if constexpr (LATE) {  // 64 rows a wave: the rows the first pass left, found by a ballot
        for (int64_t g0 = rs.g_lo + ((int64_t)blockIdx.x * 4 + wid) * 64; g0 < G; g0 += (int64_t)gridDim.x * 256) {
            const int64_t gl = g0 + lane;
            bool late = false;
            if (gl < G) {
                const int64_t r = row_rec[gl];
                late = rand_pre_slot(P, r, (uint32_t)(gl - row_off[r])) < 0;
            }
            uint32_t *const rw = s_rw[LATE ? wid : 0];
            uint32_t *const bits = rw + 4 * NXS;
            for (uint64_t m = __ballot(late); m;) {
                // up to 4 of them: group q of 16 lanes walks the q-th
                const int nr = __popcll(m) < 4 ? __popcll(m) : 4;
                uint64_t mm = m;
                for (int q = 0; q < (lane >> 4) && mm; ++q) mm &= mm - 1;
                const int64_t gq = g0 + (mm ? __builtin_ctzll(mm) : 0);
                uint64_t rec = 0;
                uint32_t kq = 0;
                if ((lane >> 4) < nr) {
                    const int64_t r = row_rec[gq];
                    rec = P.first_record + (uint64_t)r;
                    kq = (uint32_t)(gq - row_off[r]);
                }
                rand_rows16(P, nr, rec, kq, rw, bits, BW, lane);
                for (int q = 0; q < nr; ++q, m &= m - 1)
                    row_one<MR, RM1, LATE>(P, tok, rec_tok, rec_cnt, row_off, row_rec, g0 + __builtin_ctzll(m), G, out,
                                           bits + BW * q, lane);
                __builtin_amdgcn_wave_barrier();  // (the LDS is rewritten by the next rows)
            }
        }
    } else {
        for (int64_t g = rs.g_lo + (int64_t)blockIdx.x * 4 + wid; g < g_end; g += (int64_t)gridDim.x * 4)
            row_one<MR, RM1, LATE>(P, tok, rec_tok, rec_cnt, row_off, row_rec, g, G, out, nullptr, lane);
    }
}

template <int MR>  // 0: no rows; else the call's rows too (d.rows: Philox mlm / clm)
__global__ __launch_bounds__(SCAN_SMALL_NT) void k_downstream_small(SmallDown d, RowParams P,
                                                                    const uint64_t *__restrict__ off, int64_t R,
                                                                    int64_t N, int64_t n_chunks) {
    __shared__ uint32_t scratch[SCAN_SMALL_NT / 64];
    block_scan_small(d.chunk_cnt, n_chunks, d.chunk_off, scratch);
    __syncthreads();
    for (int64_t cb = (int64_t)(threadIdx.x >> 6) * COMPACT_CPW; cb < n_chunks;
         cb += (int64_t)(SCAN_SMALL_NT / 64) * COMPACT_CPW)
        compact_wave(cb, d.tokc, d.chunk_cnt, d.chunk_off, n_chunks, d.tok, d.long_count, d.chunk_ent, d.long_list,
                     d.long_scratch, d.long_pool, d.stride);
    for (int64_t r = threadIdx.x; r < R; r += SCAN_SMALL_NT)
        record_one(P, off, r, N, d.chunk_off, n_chunks, d.rec_local, d.rec_tok, d.rec_cnt, d.rec_rows);
    __syncthreads();
    block_scan_small(d.rec_rows, R, d.row_off, scratch);
    __syncthreads();
    for (int64_t r = threadIdx.x; r < R; r += SCAN_SMALL_NT)
        for (uint32_t g = d.row_off[r]; g < d.row_off[r + 1]; ++g) d.row_rec[g] = (uint32_t)r;
    if (d.stat) {
        for (int64_t r = threadIdx.x; r <= R; r += SCAN_SMALL_NT) d.stat[r] = d.row_off[r];
        if (threadIdx.x == 0) {
            d.stat[R + 1] = 0u;
            d.stat[R + 2] = d.tok_err ? *d.tok_err : 0u;  // a t5 tokenizer under mlm / clm
        }
    }
    if constexpr (MR > 0) {  // the rows, a wave each (k_rows' body), without a launch of their own
        __syncthreads();  // (this workgroup's row_off / row_rec / rec_* / ids are visible)
        const int64_t G = (int64_t)d.row_off[R];
        const int64_t g_end = d.out.direct.cap ? G : (G + P.B - 1) / P.B * P.B;
        for (int64_t g = (int64_t)(threadIdx.x >> 6); g < g_end; g += SCAN_SMALL_NT / 64)
            row_one<MR, false, false>(P, d.tok, d.rec_tok, d.rec_cnt, d.row_off, d.row_rec, g, G, d.out, nullptr,
                                      lane_id());
    }
}

template <int MR>
__global__ __launch_bounds__(64) void k_downstream_tiny(SmallDown d, RowParams P, const uint64_t *__restrict__ off,
                                                        int64_t R, int64_t N, int64_t n_chunks) {
    downstream_tiny<MR>(d, P, off, R, N, n_chunks);
}

hipError_t launch_downstream_small(const SmallDown &d, const RowParams &P, const uint64_t *off, int64_t R, int64_t N,
                                   hipStream_t st) {
    const int64_t n_chunks = (N + CHUNK - 1) / CHUNK;
    if (n_chunks > SMALL_CHUNKS || R > SCAN_SMALL) return hipErrorInvalidValue;
    const int MR = (P.S + 255) / 256;
    if (d.rows && ((P.rng_mode == 1 && P.task == 0) || (P.task != 0 && P.task != 1)))
        return hipErrorInvalidValue;  // (rng_mode 1 masks need k_rows' passes; span has its own rows)
    const bool tiny = R <= 64 && n_chunks <= 64;
#define LAUNCH_DS(M)                                                                                                    \
    if (tiny) hipLaunchKernelGGL(k_downstream_tiny<M>, dim3(1), dim3(64), 0, st, d, P, off, R, N, n_chunks);        \
    else hipLaunchKernelGGL(k_downstream_small<M>, dim3(1), dim3(SCAN_SMALL_NT), 0, st, d, P, off, R, N, n_chunks)
    if (!d.rows) LAUNCH_DS(0);
    else if (MR <= 1) LAUNCH_DS(1);
    else if (MR <= 2) LAUNCH_DS(2);
    else if (MR <= 4) LAUNCH_DS(4);
    else if (MR <= 8) LAUNCH_DS(8);
    else return hipErrorInvalidValue;
#undef LAUNCH_DS
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// rand-compatible MLM masks (rng_mode 1, oracle/orc_batcher.c orc_rand_positions):
// BertData::mask_batch's position_base.shuffle (bert_data.rs:40-43; rand 0.8.5
// SliceRandom::shuffle -> gen_index -> UniformInt<u32>::sample_single_inclusive)
// driven by StdRng::from_seed(seed | record | chunk) (rand_chacha 0.3.1 ChaCha12:
// 64-bit block counter, stream 0, words in block order).
// The draws are sequential: swap i = S-1 .. 1 takes words until one is
// accepted, lo32(v * n) <= zone(n) = (n << lz(n)) - 1 with n = i + 1 -- rand's
// "conservative" zone rejects up to half the words for n just above a power of
// two, so about 30 % of a row's ~730 words are rejected and every row has
// rejections.  Phase A runs each row's walk in one lane: the lane computes its
// ChaCha12 blocks in registers, 16 words per block in an unrolled loop, and writes
// each swap index j_i to the row's slice of `jbuf`; the walk stops after step k
// (steps k-1 .. 1 only permute [0, k) among itself).  A row is keyed by (seed,
// record, chunk) alone, so the chunk-0 row of every record (86 % of the bench's
// rows) is walked by k_mask_rand_rec (64 records per wave) on a second stream beside
// the tokenizer, and phase B (k_mask_bits_rec) turns them into mask bits there too;
// k_rows<MR, true> reads the bits, and walks the few rows left (chunk >= 1 past the
// byte-length guess) in a second pass (rand_rows16).  Phase B (rand_set_bits), a
// wave per row: mask_batch only uses the SET of the first k shuffled
// positions, and Fisher-Yates from the end never moves a value out of [0, k)
// once steps i < k begin (j_i <= i), so the set is what [0, k) holds after steps
// S-1 .. k.  The value at position p just before step p came from the latest
// earlier swap into p -- step next(p) = min{i > p : j_i = p, j_i != i} -- so it
// is val(next(p)), or p; [0, k) receives val(min{i >= k : j_i = x}) at each x.
// next() is one LDS atomicMin per step; each x follows a chain of ~2 hops
// (S=512, k=76).  Output: the row's mask bits.
// ---------------------------------------------------------------------------
// Phase A, NR rows per lane: row r of the lane is (rec[r], chunk[r]) when active[r]; writes its
// swap indices j_i, i = S-1 .. k, to jrow[r].  Every lane of the wave calls it (the block loop is
// wave-uniform).  The rows' ChaCha12 rounds and acceptance chains are independent, so NR > 1
// gives the scheduler NR-fold ILP: a lane's walk is a chain of dependent 64-bit multiplies and
// selects, and one row per lane leaves the SIMD waiting on it.
template <int NR>
__device__ __forceinline__ void rand_walk_lanes(const RowParams &P, const bool (&active)[NR], const uint64_t (&rec)[NR],
                                                const uint32_t (&chunk)[NR], uint16_t *const (&jrow)[NR]) {
    const int S = P.S, kmask = P.mask_length < S ? P.mask_length : S;
    // only steps i >= k move values into or out of [0, k): the walk stops there
    const int i0 = kmask > 1 ? kmask : 1;
    int i[NR];
    uint32_t n[NR], zone[NR];
    ChaRow cr[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        uint32_t key[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
        i[r] = 0;
        if (active[r]) {
            key[0] = (uint32_t)P.seed;
            key[1] = (uint32_t)(P.seed >> 32);
            key[2] = (uint32_t)rec[r];
            key[3] = (uint32_t)(rec[r] >> 32);
            key[4] = chunk[r];
            i[r] = S - 1;
        }
        chacha_row_init(cr[r], key);
        n[r] = (uint32_t)i[r] + 1u;
        zone[r] = (n[r] << __builtin_clz(n[r])) - 1u;
    }
    // (S % 8 == 0) indices are collected eight at a time -- positions 8b .. 8b + 7, the
    // walk runs downwards -- in a 128-bit shift register and stored as one 16-B store:
    // a lane's own row, so each per-index 2-B store would touch its own line
    const bool vec = (S & 7) == 0;
    uint32_t a0[NR], a1[NR], a2[NR], a3[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) a0[r] = a1[r] = a2[r] = a3[r] = 0u;
    auto live = [&] {
        bool x = false;
#pragma unroll
        for (int r = 0; r < NR; ++r) x |= i[r] >= i0;
        return x;
    };
    for (uint32_t blk = 0; __any(live()); ++blk) {
        uint32_t o[NR][16];
#pragma unroll
        for (int r = 0; r < NR; ++r) chacha12_block_row(cr[r], blk, o[r]);
        if (vec) {
            // branch-free per word (selects, no exec-mask work on the one scalar unit per
            // CU); only the store of a completed group of eight is predicated
#pragma unroll
            for (int q = 0; q < 16; ++q)
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const uint64_t m = (uint64_t)o[r][q] * n[r];
                    const bool acc = i[r] >= i0 && (uint32_t)m <= zone[r];
                    const uint32_t v = (uint32_t)(m >> 32);
                    a3[r] = acc ? (a3[r] << 16) | (a2[r] >> 16) : a3[r];
                    a2[r] = acc ? (a2[r] << 16) | (a1[r] >> 16) : a2[r];
                    a1[r] = acc ? (a1[r] << 16) | (a0[r] >> 16) : a1[r];
                    a0[r] = acc ? (a0[r] << 16) | v : a0[r];
                    if (acc && (i[r] & 7) == 0)  // positions i .. i + 7 are complete
                        *reinterpret_cast<uint4 *>(jrow[r] + i[r]) = make_uint4(a0[r], a1[r], a2[r], a3[r]);
                    i[r] -= acc ? 1 : 0;
                    n[r] = (uint32_t)i[r] + 1u;
                    zone[r] = (n[r] << __builtin_clz(n[r])) - 1u;
                }
        } else {
#pragma unroll
            for (int q = 0; q < 16; ++q)
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const uint64_t m = (uint64_t)o[r][q] * n[r];
                    if (i[r] >= i0 && (uint32_t)m <= zone[r]) {
                        jrow[r][i[r]] = (uint16_t)(m >> 32);
                        --i[r];
                        n[r] = (uint32_t)i[r] + 1u;
                        zone[r] = (n[r] << __builtin_clz(n[r])) - 1u;
                    }
                }
        }
    }
#pragma unroll
    for (int r = 0; r < NR; ++r)
        if (vec && active[r] && (i0 & 7) != 0) {  // the partial block [i0, (i0 | 7)]
            const uint32_t w[4] = {a0[r], a1[r], a2[r], a3[r]};
            for (int p = i0; p <= (i0 | 7); ++p) {  // position p is the (p - i0)-th newest value
                const int d = p - i0;
                jrow[r][p] = (uint16_t)(w[d >> 1] >> (16 * (d & 1)));
            }
        }
}

// Phase B for one row, one wave: jr = the row's swap indices -> its mask bits in bt
// (ceil(S/32) words of the wave's LDS; nx: 64 * MR words, MR >= S / 64)
template <int MR>
__device__ __forceinline__ void rand_set_bits(const RowParams &P, const uint16_t *__restrict__ jr, uint32_t *nx,
                                              uint32_t *bt, int lane) {
    const int S = P.S, kmask = P.mask_length < S ? P.mask_length : S;
    const int i0 = kmask > 1 ? kmask : 1;
    constexpr uint32_t NONE = 0xFFFFFFFFu;
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
    uint32_t jc[MR];
#pragma unroll
    for (int m = 0; m < MR; ++m) {
        const int t = lane + 64 * m;
        jc[m] = t >= i0 && t < S ? (uint32_t)jr[t] : (uint32_t)t;  // (t, t): no move
    }
#pragma unroll
    for (int m = 0; m < MR; ++m) nx[lane + 64 * m] = NONE;
    if (lane < 2 * MR) bt[lane] = 0u;
    wave_sync();
    // next(p): the latest swap into p among steps i >= k (a self swap moves nothing)
#pragma unroll
    for (int m = 0; m < MR; ++m)
        if (jc[m] != (uint32_t)(lane + 64 * m)) atomicMin(&nx[jc[m]], (uint32_t)(lane + 64 * m));
    wave_sync();
    // [0, k) holds val(next(x)) (or x): follow each chain to its end
    for (int x = lane; x < kmask; x += 64) {
        uint32_t p = (uint32_t)x;
        for (uint32_t q = nx[p]; q != NONE; q = nx[p]) p = q;
        atomicOr(&bt[p >> 5], 1u << (p & 31));
    }
    wave_sync();
}

// Chunk-0 rows, RAND_NR records per lane, 64 RAND_NR per wave: the walk (rand_walk_lanes) keyed
// by (first_record + r, chunk 0) -- which needs nothing the tokenizer computes, so the host runs
// it on a second stream beside the tokenizer (sdl_batcher.cpp run_device): its ChaCha12 work
// fills VALU slots the latency-bound tokenizer leaves idle instead of sitting on the step's
// critical path.  (86 % of the bench's rows are chunk 0.)
// (slot s < R: record s, chunk 0; s = R + i: chunk 1 of the list's i-th record, the records of
// >= mask_spec1 bytes, in no particular order; mask_spos[r] = i.)  The walk runs over the slots
// t in [0, R + n_spec) -- a wave holding any chunk-1 slot costs a whole walk, and ~1 record in 5
// has one -- and the slots take R + (the records past mask_spec1 bytes), not 2 R, of the buffers.
__global__ __launch_bounds__(256) void k_rand_spec_list(RowParams P, uint32_t *__restrict__ list,
                                                        uint32_t *__restrict__ spos) {
    const int lane = lane_id();
    const int64_t R = P.mask_R;
    for (int64_t r0 = (int64_t)blockIdx.x * 256 + (threadIdx.x & ~63u); r0 < R; r0 += (int64_t)gridDim.x * 256) {
        const int64_t r = r0 + lane;
        const bool take = r < R && (int64_t)(P.mask_off[r + 1] - P.mask_off[r]) >= P.mask_spec1;
        const uint64_t m = __ballot(take);
        if (!m) continue;
        const int leader = __builtin_ctzll(m);
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&list[0], (uint32_t)__popcll(m));
        base = (uint32_t)lane_bcast((int)base, leader);
        if (take) {
            const uint32_t i = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            list[1 + i] = (uint32_t)r;
            spos[r] = i;
        }
    }
}
// record of slot t (chunk 0 below R, chunk 1 above)
__device__ __forceinline__ int64_t rand_rec_of(const RowParams &P, const uint32_t *list, int64_t t) {
    return t < P.mask_R ? t : (int64_t)list[1 + (t - P.mask_R)];
}
constexpr int RAND_NR = 1;  // rows per lane in k_mask_rand_rec
__global__ __launch_bounds__(256) void k_mask_rand_rec(RowParams P, const uint32_t *__restrict__ list,
                                                       uint16_t *__restrict__ jbuf) {
    const int lane = lane_id();
    const int64_t R = P.mask_R, nt = R + (P.mask_spec1 > 0 ? (int64_t)list[0] : 0);
    const int64_t waves = (int64_t)gridDim.x * 4;
    constexpr int64_t W = 64 * RAND_NR;
    for (int64_t t0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * W; t0 < nt; t0 += waves * W) {
        bool active[RAND_NR];
        uint64_t rec[RAND_NR];
        uint32_t chunk[RAND_NR];
        uint16_t *jrow[RAND_NR];
#pragma unroll
        for (int r = 0; r < RAND_NR; ++r) {
            const int64_t t = t0 + 64 * r + lane;
            active[r] = t < nt;
            const int64_t s = active[r] ? t : 0;
            rec[r] = P.first_record + (uint64_t)(active[r] ? rand_rec_of(P, list, t) : 0);
            chunk[r] = s < R ? 0u : 1u;
            jrow[r] = jbuf + s * (int64_t)P.S;
        }
        rand_walk_lanes<RAND_NR>(P, active, rec, chunk, jrow);
    }
}

// Phase B for those rows: a wave per row, its mask bits -> bits[slot]
template <int MR4>
__global__ __launch_bounds__(256) void k_mask_bits_rec(RowParams P, const uint32_t *__restrict__ list,
                                                       const uint16_t *__restrict__ jbuf, uint32_t *__restrict__ bits) {
    __shared__ uint32_t s_nx[4][64 * MR4];
    __shared__ uint32_t s_bt[4][2 * MR4];
    const int lane = lane_id(), wid = (int)(threadIdx.x >> 6);
    const int64_t nt = P.mask_R + (P.mask_spec1 > 0 ? (int64_t)list[0] : 0);
    for (int64_t t = (int64_t)blockIdx.x * 4 + wid; t < nt; t += (int64_t)gridDim.x * 4) {
        const int64_t s = t;
        rand_set_bits<MR4>(P, jbuf + s * (int64_t)P.S, s_nx[wid], s_bt[wid], lane);
        for (int w = lane; w < P.mask_w; w += 64) bits[s * (int64_t)P.mask_w + w] = s_bt[wid][w];
        __builtin_amdgcn_wave_barrier();  // (s_bt is rewritten by the wave's next row)
    }
}

hipError_t launch_mask_rand_rec(const RowParams &P, uint32_t *list, uint32_t *spos, uint16_t *jbuf, uint32_t *bits,
                                hipStream_t st) {
    const int64_t R = P.mask_R, ns = P.mask_spec1 > 0 ? 2 * R : R;
    if (R <= 0) return hipSuccess;
    if (P.S > RAND_MAX_S || P.mask_w * 32 < P.S || !P.mask_off) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(list, 0, 4, st);
    if (e != hipSuccess) return e;
    if (P.mask_spec1 > 0) {
        const int64_t lb = (R + 255) / 256;
        hipLaunchKernelGGL(k_rand_spec_list, dim3((unsigned)(lb < 2048 ? lb : 2048)), dim3(256), 0, st, P, list, spos);
    }
    // (sized for every slot; the waves past R + n_spec leave at once)
    const int64_t want = (ns + 256 * RAND_NR - 1) / (256 * RAND_NR);
    hipLaunchKernelGGL(k_mask_rand_rec, dim3((unsigned)(want < 4096 ? want : 4096)), dim3(256), 0, st, P,
                       (const uint32_t *)list, jbuf);
    const int64_t wb = (ns + 3) / 4;
    const dim3 g((unsigned)(wb < 16384 ? wb : 16384));
    const int MR4 = (P.S + 63) / 64;
#define LAUNCH_BITS(M) hipLaunchKernelGGL(k_mask_bits_rec<M>, g, dim3(256), 0, st, P, (const uint32_t *)list, (const uint16_t *)jbuf, bits)
    if (MR4 <= 2) LAUNCH_BITS(2);
    else if (MR4 <= 4) LAUNCH_BITS(4);
    else if (MR4 <= 8) LAUNCH_BITS(8);
    else if (MR4 <= 16) LAUNCH_BITS(16);
    else LAUNCH_BITS(32);
#undef LAUNCH_BITS
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// The host path's D2H: one launch copies every segment's rows of all planes
// straight into the batches' pinned blocks (device-mapped host memory), 16-B
// stores per lane, instead of one hipMemcpyAsync per plane per batch segment.
// Block (seg, y) copies rows y, y + gridDim.y, ... of segment seg; its four
// waves take the four planes.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_rows_to_host(const RowSeg *__restrict__ segs, const int32_t *__restrict__ ids,
                                                      const int32_t *__restrict__ am, const int32_t *__restrict__ tt,
                                                      const int32_t *__restrict__ lab, int S, int LW) {
    const RowSeg sg = segs[blockIdx.x];
    const int plane = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    const int32_t *src = plane == 0 ? ids : plane == 1 ? am : plane == 2 ? tt : lab;
    int32_t *dst = plane == 0 ? sg.ids : plane == 1 ? sg.am : plane == 2 ? sg.tt : sg.lab;
    if (!src || !dst) return;
    const int W = plane == 3 ? LW : S;  // ints per row
    const bool vec = (W & 3) == 0;
    for (uint32_t r = blockIdx.y; r < sg.n; r += gridDim.y) {
        const int32_t *s = src + (size_t)(sg.g0 + r) * W;
        int32_t *d = dst + (size_t)(sg.dst + r) * W;
        if (vec) {
            for (int j = 4 * lane; j < W; j += 256)
                *reinterpret_cast<int4 *>(d + j) = *reinterpret_cast<const int4 *>(s + j);
        } else {
            for (int j = lane; j < W; j += 64) d[j] = s[j];
        }
    }
}

hipError_t launch_rows_to_host(const RowSeg *segs, int n_segs, uint32_t rows_per_seg_max, const int32_t *ids,
                               const int32_t *am, const int32_t *tt, const int32_t *lab, int S, int LW,
                               hipStream_t st) {
    if (n_segs <= 0) return hipSuccess;
    const unsigned gy = rows_per_seg_max < 64u ? (rows_per_seg_max ? rows_per_seg_max : 1u) : 64u;
    hipLaunchKernelGGL(k_rows_to_host, dim3((unsigned)n_segs, gy), dim3(256), 0, st, segs, ids, am, tt, lab, S, LW);
    return hipGetLastError();
}

// (kernels.hpp DirectDst) block b copies rows b, b + gridDim.x, ... below
// min(row_off[R], cap), its four waves taking the four planes; block 0 also
// copies the row offsets and error words out.
__global__ __launch_bounds__(256) void k_rows_direct(DirectDst d, const uint32_t *__restrict__ row_off, int64_t R,
                                                     const int32_t *__restrict__ ids, const int32_t *__restrict__ am,
                                                     const int32_t *__restrict__ tt, const int32_t *__restrict__ lab,
                                                     int S, int LW, const uint32_t *__restrict__ err0,
                                                     const uint32_t *__restrict__ err1, uint32_t *__restrict__ stat) {
    if (blockIdx.x == 0) {
        for (int64_t r = threadIdx.x; r <= R; r += 256) stat[r] = row_off[r];
        if (threadIdx.x == 0) {
            stat[R + 1] = err0 ? *err0 : 0u;
            stat[R + 2] = err1 ? *err1 : 0u;
        }
    }
    const uint32_t total = row_off[R];
    const uint32_t n = total < d.cap ? total : d.cap;
    const int plane = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    const int32_t *src = plane == 0 ? ids : plane == 1 ? am : plane == 2 ? tt : lab;
    if (!src) return;
    const int W = plane == 3 ? LW : S;  // ints per row
    const bool vec = (W & 3) == 0;
    for (uint32_t g = blockIdx.x; g < n; g += gridDim.x) {
        const uint32_t slot = d.base + g, bi = slot >= d.B ? 1u : 0u, row = slot - bi * d.B;
        int32_t *dst = plane == 0 ? d.ids[bi] : plane == 1 ? d.am[bi] : plane == 2 ? d.tt[bi] : d.lab[bi];
        const int32_t *s = src + (size_t)g * W;
        int32_t *o = dst + (size_t)row * W;
        if (vec) {
            for (int j = 4 * lane; j < W; j += 256)
                *reinterpret_cast<int4 *>(o + j) = *reinterpret_cast<const int4 *>(s + j);
        } else {
            for (int j = lane; j < W; j += 64) o[j] = s[j];
        }
    }
}

hipError_t launch_rows_direct(const DirectDst &d, const uint32_t *row_off, int64_t R, const int32_t *ids,
                              const int32_t *am, const int32_t *tt, const int32_t *lab, int S, int LW,
                              const uint32_t *err0, const uint32_t *err1, uint32_t *stat, hipStream_t st) {
    const unsigned grid = d.cap < 64u ? (d.cap ? d.cap : 1u) : 64u;
    hipLaunchKernelGGL(k_rows_direct, dim3(grid), dim3(256), 0, st, d, row_off, R, ids, am, tt, lab, S, LW, err0, err1,
                       stat);
    return hipGetLastError();
}

hipError_t launch_rows(const RowParams &P, const uint32_t *tok, const uint32_t *rec_tok, const uint32_t *rec_cnt,
                       const uint32_t *row_off, const uint32_t *row_rec, SegSel sel, int64_t rows_cap, RowOut out,
                       hipStream_t st, hipStream_t st_late) {
    if (!st_late) st_late = st;
    if (rows_cap == 0) return hipSuccess;
constexpr int ROWS_GRID_CAP = 16384;
    const int64_t want = (rows_cap + 3) / 4;
    const unsigned grid = (unsigned)(want < ROWS_GRID_CAP ? want : ROWS_GRID_CAP);
    const int MR = (P.S + 255) / 256;
    if (P.label_width > 256 * MR) return hipErrorInvalidValue;
    const bool rm1 = P.task == 0 && P.rng_mode == 1;
    if (rm1 && ((P.mask_bits0 && !P.mask_off) || P.mask_w * 32 < P.S || P.S > RAND_MAX_S))
        return hipErrorInvalidValue;
    // (rng_mode 1: the late pass scans 256 rows a block)
    const int64_t want_late = (rows_cap + 255) / 256;
    const unsigned grid_late = (unsigned)(want_late < 2048 ? want_late : 2048);
#define LAUNCH_ROWS(MM)                                                                                                 \
    if (rm1) {                                                                                                        \
        hipLaunchKernelGGL((k_rows<MM, true>), dim3(grid), dim3(256), 0, st, P, tok, rec_tok, rec_cnt, row_off,      \
                           row_rec, sel, rows_cap, out);                                                              \
        hipLaunchKernelGGL((k_rows<MM, true, true>), dim3(grid_late), dim3(256), 0, st_late, P, tok, rec_tok, rec_cnt, \
                           row_off, row_rec, sel, rows_cap, out);                                                     \
    } else                                                                                                            \
        hipLaunchKernelGGL((k_rows<MM, false>), dim3(grid), dim3(256), 0, st, P, tok, rec_tok, rec_cnt, row_off,     \
                           row_rec, sel, rows_cap, out)
    if (MR <= 1) LAUNCH_ROWS(1);
    else if (MR <= 2) LAUNCH_ROWS(2);
    else if (MR <= 4) LAUNCH_ROWS(4);
    else if (MR <= 8) LAUNCH_ROWS(8);
    else return hipErrorInvalidValue;
#undef LAUNCH_ROWS
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// T5Data::put_data (models/t5_data.rs:162-226) for every row, task=span.
// A row is one chunk of n <= S framed ids.  Pass p draws gap g_p and span size
// s_p; because the input cursor never passes the id cursor (lp <= ip <= n <= S),
// the only clamp that binds is n - ip, and only in the last pass (the first
// whose g + s reaches n).  One wave per row, in rounds of up to 64 passes:
//   A. lanes take passes: each lane's draws, then wave prefix sums give every
//      pass's id cursor I_p, input cursor lp_p = I_p - A_p + p (A_p = ids
//      spanned before p) and label cursor ap_p = A_p + p; the ballot finds
//      the last pass; the round's pass records go to LDS;
//   B. the planes are written position-parallel (lane = position, coalesced
//      stores): a position's pass is the last one starting at or before it
//      (a scalar walk over the few pass starts inside each 64-position group),
//      and its value is a gap id, the sentinel, or a spanned id.
// Draws: rng_mode 0 = the RNG contract (Philox(p, chunk | 1 << 30, record;
// seed) words 0/1 through the CDF tables); rng_mode 1 = the reference's
// random_data_gap / random_data_size on the row's StdRng (span_draws_rand).
// Labels past the S/4 label width (the reference panics) are skipped and
// counted in *err; so is a sentinel index >= 100 (extra[99] is written).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t span_pick(int32_t kmin, int32_t n, const uint32_t (&thr)[32], uint32_t x) {
    int32_t v = kmin;
#pragma unroll
    for (int j = 0; j < 32; ++j) v += (j < n && thr[j] <= x) ? 1 : 0;
    return (uint32_t)v;
}

// ---- rng_mode 1: rand_distr 0.4.3 StandardNormal (f64) on the row's StdRng ----
// (oracle/orc_batcher.c std_normal).  utils::ziggurat: bits = next_u64,
// i = bits & 0xff, u = [2,4) float of bits >> 12 minus 3, x = u * X[i];
// |x| < X[i+1] returns x (~99 % of draws, one u64); i == 0 takes the tail
// (pairs of Open01 until -2 ln c >= (ln a / R)^2); else the wedge test with
// one more u64.  The row's stream: u64 k = ChaCha12 words 2k (low), 2k+1.
constexpr int SPAN_WBLK = 17;             // ChaCha12 blocks per window (lanes 0..16)
constexpr int SPAN_WU64 = 8 * SPAN_WBLK;  // 136 u64 draws-worth of stream per window
constexpr double ZIG_R = 3.6541528853610088;

struct SpanStream {
    uint32_t key[8];
    const uint32_t *win;  // LDS: blocks [wblk, wblk + SPAN_WBLK)
    uint64_t wblk;
    uint32_t cblk[16];    // one block computed beyond the window (rare)
    int64_t chave;
    __device__ uint64_t at(uint64_t k) {
        const uint64_t b = k >> 3;
        uint32_t lo, hi;
        if (b - wblk < (uint64_t)SPAN_WBLK) {
            const uint32_t w = (uint32_t)(2 * (k - 8 * wblk));
            lo = win[w];
            hi = win[w + 1];
        } else {
            if ((int64_t)b != chave) {
                chacha12_block(key, (uint32_t)b, cblk);
                chave = (int64_t)b;
            }
            lo = cblk[2 * (k & 7)];
            hi = cblk[2 * (k & 7) + 1];
        }
        return (uint64_t)hi << 32 | lo;
    }
};

__device__ __forceinline__ double bits_f64(uint64_t b) { return __longlong_as_double((long long)b); }

// the ziggurat's fast exit for the draw starting with `bits` (x in *x)
__device__ __forceinline__ bool zig_fast(uint64_t bits, const double *__restrict__ ZX, double *x) {
#pragma clang fp contract(off)
    const int i = (int)(bits & 0xffu);
    const double u = bits_f64((bits >> 12) | (1024ull << 52)) - 3.0;
    *x = u * ZX[i];
    return fabs(*x) < ZX[i + 1];
}

// The whole draw starting at stream word k: value and u64 words consumed.
template <class Stream>
__device__ double zig_normal(Stream &s, uint64_t k, const double *__restrict__ ZX,
                             const double *__restrict__ ZF, uint32_t *len) {
#pragma clang fp contract(off)
    const uint64_t k0 = k;
    for (;;) {
        const uint64_t bits = s.at(k++);
        const int i = (int)(bits & 0xffu);
        const double u = bits_f64((bits >> 12) | (1024ull << 52)) - 3.0;
        const double x = u * ZX[i];
        if (fabs(x) < ZX[i + 1]) {
            *len = (uint32_t)(k - k0);
            return x;
        }
        if (i == 0) {  // zero_case
            double xt = 1.0, yt = 0.0;
            while (-2.0 * yt < xt * xt) {
                const double a = bits_f64((s.at(k++) >> 12) | (1023ull << 52)) - (1.0 - 0x1p-53);
                const double c = bits_f64((s.at(k++) >> 12) | (1023ull << 52)) - (1.0 - 0x1p-53);
                xt = log(a) / ZIG_R;
                yt = log(c);
            }
            *len = (uint32_t)(k - k0);
            return u < 0.0 ? xt - ZIG_R : ZIG_R - xt;
        }
        const double g = (double)(s.at(k++) >> 11) * 0x1p-53;
        if (ZF[i + 1] + (ZF[i] - ZF[i + 1]) * g < exp(-x * x / 2.0)) {
            *len = (uint32_t)(k - k0);
            return x;
        }
    }
}

// `f as usize` (saturating; NaN and negatives 0), then min with n
__device__ __forceinline__ uint32_t sat_draw(double d, int n) {
    if (!(d > 0.0)) return 0u;
    return d >= (double)n ? (uint32_t)n : (uint32_t)d;
}

// The round's draws (up to 128 = 64 passes) from stream word *spos on:
// lanes compute the window's blocks and test every draw start for the fast
// exit; a wave-uniform walk over the rare slow starts (each one's length from
// the lane that owns it) finds which words start draws; draw d lands in
// s_draw[d].  Returns the draws this round can use (even, >= 2) and advances
// *spos past them.
__device__ int span_draws_rand(SpanStream &s, uint64_t *spos, const double *__restrict__ ZX,
                               const double *__restrict__ ZF, uint32_t *s_win, double *s_draw, uint16_t *s_dend) {
    const int lane = lane_id();
    const uint64_t p0 = *spos;
    s.wblk = p0 >> 3;
    s.chave = -1;
    s.win = s_win;
    if (lane < SPAN_WBLK) {
        uint32_t o[16];
        chacha12_block(s.key, (uint32_t)(s.wblk + (uint64_t)lane), o);
#pragma unroll
        for (int q = 0; q < 16; ++q) s_win[16 * lane + q] = o[q];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // offsets o = lane, lane + 64 from p0: fast exit or the full draw
    double v[2];
    uint32_t L[2];
    bool slow[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        slow[h] = !zig_fast(s.at(p0 + (uint64_t)(lane + 64 * h)), ZX, &v[h]);
        L[h] = 1u;
    }
    const uint64_t m0 = __ballot(slow[0]), m1 = __ballot(slow[1]);
    if (m0 | m1) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
            if (slow[h]) v[h] = zig_normal(s, p0 + (uint64_t)(lane + 64 * h), ZX, ZF, &L[h]);
    }
    // which offsets start draws: fast runs between slow starts; a slow start
    // at o covers o .. o + L(o) - 1
    uint64_t mem0 = ~0ull, mem1 = ~0ull;
    uint32_t cur = 0;
    uint64_t q0 = m0, q1 = m1;
    while (q0 | q1) {
        const uint32_t sl = q0 ? (uint32_t)__builtin_ctzll(q0) : 64u + (uint32_t)__builtin_ctzll(q1);
        const uint32_t Ls = sl < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)L[0], (int)sl)
                                    : (uint32_t)__builtin_amdgcn_readlane((int)L[1], (int)(sl - 64));
        const uint32_t nxt = sl + Ls;  // offsets sl + 1 .. nxt - 1 are consumed by this draw
        for (uint32_t o = sl + 1; o < nxt && o < 128u; ++o) {  // (few words: a wedge test adds one)
            if (o < 64) mem0 &= ~(1ull << o); else mem1 &= ~(1ull << (o - 64));
        }
        cur = nxt;
        if (cur >= 128u) break;
        // the next slow start at or after cur
        q0 = cur < 64 ? m0 & (~0ull << cur) : 0ull;
        q1 = cur < 64 ? m1 : (cur < 128 ? m1 & (~0ull << (cur - 64)) : 0ull);
    }
    (void)cur;
    // draw numbers: members below each offset; draw d ends (relative) at o + L
    const int n0 = __builtin_popcountll(mem0);
    const int D = n0 + __builtin_popcountll(mem1);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint64_t mm = h ? mem1 : mem0;
        if ((mm >> lane) & 1ull) {
            const int d = (h ? n0 : 0) + __builtin_popcountll(mm & ((1ull << lane) - 1ull));
            s_draw[d] = v[h];
            s_dend[d] = (uint16_t)(lane + 64 * h + (int)L[h]);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    int nd = D & ~1;
    if (nd == 0) {  // (a slow draw at offset 0 ran past offset 128) one pass, drawn in order
        if (lane == 0) {
            uint32_t l1, l2;
            s_draw[0] = zig_normal(s, p0, ZX, ZF, &l1);
            s_draw[1] = zig_normal(s, p0 + l1, ZX, ZF, &l2);
            s_dend[1] = (uint16_t)(l1 + l2);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        nd = 2;
    }
    return nd;
}

struct SpanPass {  // one pass of a round (LDS): cursors and lengths
    uint32_t lp_gg;   // input cursor | gap ids written << 16
    uint32_t ip_sz;   // id cursor | spanned ids written << 16
    uint32_t ap;      // label cursor
    uint32_t pass;    // pass index in the row
};

__device__ __forceinline__ void st_nt(int32_t *p, int32_t v) { __builtin_nontemporal_store(v, p); }

constexpr int SPAN_WAVES = 6;  // (RAND 0) 75 VGPRs, no spills: 0.507 -> 0.428 ms; 7 and 8 spill
constexpr int SPAN_GRID_CAP = 16384;  // with 6 waves per SIMD: 0.428 -> 0.414 ms
template <int RAND>  // draws: 0 the Philox contract, 1 the row's StdRng (rng_mode 1)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RAND ? 1 : SPAN_WAVES, 8))) void k_rows_span(RowParams P, const uint32_t *__restrict__ tok,
                                                   const uint32_t *__restrict__ rec_tok,
                                                   const uint32_t *__restrict__ rec_cnt,
                                                   const uint32_t *__restrict__ row_off,
                                                   const uint32_t *__restrict__ row_rec, SegSel sel,
                                                   int64_t rows_cap, RowOut out, uint32_t *__restrict__ err,
                                                   const uint32_t *__restrict__ list,
                                                   const uint32_t *__restrict__ list_n) {
    __shared__ SpanPass s_pass[4][64];
    __shared__ uint32_t s_win[4][SPAN_WBLK * 16];
    __shared__ double s_draw[4][128];
    __shared__ uint16_t s_dend[4][128];
    __shared__ int32_t s_extra[100];    // <extra_id_0..99>: a sentinel store reads LDS, not global memory
    extern __shared__ int32_t s_rid[];  // [4][S]: each wave's row of framed ids (dynamic)
    const int lane = lane_id();
    const int wid = (int)(threadIdx.x >> 6);
    if (threadIdx.x < 100) s_extra[threadIdx.x] = P.extra_ids[threadIdx.x];
    __syncthreads();
    const int S = P.S, LW = P.label_width;
    const RowSpan rs = row_span(sel, row_off, P.B, rows_cap);
    const int64_t G = rs.g_real;
    SpanPass *sp = s_pass[wid];
    // list mode (the two-phase path's rows with more passes than its plan holds): those rows only
    const int64_t i_end = list ? (int64_t)*list_n : rs.g_end;
    for (int64_t i = (list ? 0 : rs.g_lo) + (int64_t)blockIdx.x * 4 + wid; i < i_end; i += (int64_t)gridDim.x * 4) {
        const int64_t g = list ? (int64_t)list[i] : i;
        int32_t *ids_o = out.input_ids + g * S;
        int32_t *am_o = out.attention_mask + g * S;
        int32_t *lb_o = out.labels + g * (int64_t)LW;
        for (int j = lane; j < S; j += 64) st_nt(am_o + j, 1);  // attention stays 1 (the zeroing loop is empty)
        if (g >= (int64_t)G) {
            for (int j = lane; j < S; j += 64) st_nt(ids_o + j, 0);
            for (int j = lane; j < LW; j += 64) st_nt(lb_o + j, -100);
            continue;
        }
        const int64_t r = row_rec[g];
        const uint32_t k = (uint32_t)(g - row_off[r]);
        const uint32_t cnt = rec_cnt[r];
        const uint32_t t0 = rec_tok[r];
        const int64_t nf = (int64_t)cnt + P.n_pre + P.n_post;
        const int64_t base = P.chunk ? (int64_t)k * S : 0;
        const int n = (int)((nf - base) < S ? (nf - base) : S);
        if (n <= 0) continue;  // (a row always holds >= 1 id)
        auto fid = [&](int j) -> int32_t {  // framed id j of this chunk
            const int64_t f = base + j;
            if (f < P.n_pre) return frame_id(P.pre, (int)f);
            if (f < P.n_pre + (int64_t)cnt) return (int32_t)tok[t0 + (f - P.n_pre)];
            return frame_id(P.post, (int)(f - P.n_pre - cnt));
        };
        auto extra = [&](uint32_t q) -> int32_t { return s_extra[q < 100u ? q : 99u]; };
        // the row's framed ids into LDS first: one coalesced burst with every
        // load in flight, so the position-parallel writes below read LDS only
        int32_t *rid = s_rid + (size_t)wid * S;
        for (int j0 = 0; j0 < n; j0 += 64 * 8) {
            int32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int j = j0 + 64 * u + lane;
                v[u] = j < n ? fid(j) : 0;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int j = j0 + 64 * u + lane;
                if (j < n) rid[j] = v[u];
            }
        }
        const uint64_t rec = P.first_record + (uint64_t)r;
        SpanStream ss;
        uint64_t spos = 0;
        if (RAND) {
            const uint32_t kk[8] = {(uint32_t)P.seed, (uint32_t)(P.seed >> 32), (uint32_t)rec, (uint32_t)(rec >> 32),
                                    k, 0u, 0u, 0u};
#pragma unroll
            for (int q = 0; q < 8; ++q) ss.key[q] = kk[q];
        }
        uint32_t bad = 0;
        int I0 = 0, A0 = 0;  // ids consumed / ids spanned before this round
        int lp_end = 0, ap_end = 0;
        for (uint32_t p0 = 0;;) {
            // ---- A. this round's passes ----
            int np = 64;
            uint32_t gr, sr;
            if (RAND) {
                np = span_draws_rand(ss, &spos, P.zig_x, P.zig_f, s_win[wid], s_draw[wid], s_dend[wid]) >> 1;
                np = np < 64 ? np : 64;
                gr = sat_draw(P.avg_span_gap - s_draw[wid][2 * (lane < np ? lane : 0)], n);
                const uint32_t sz = sat_draw(P.avg_span_size - s_draw[wid][2 * (lane < np ? lane : 0) + 1], n);
                sr = sz > 1u ? sz : 1u;  // std::cmp::max(distance as usize, 1)
                spos += s_dend[wid][2 * np - 1];
            } else {
                const uint32_t p = p0 + (uint32_t)lane;
                const uint4 c = philox4x32_10(make_uint4(p, k | 0x40000000u, (uint32_t)rec, (uint32_t)(rec >> 32)),
                                              (uint32_t)P.seed, (uint32_t)(P.seed >> 32));
                gr = span_pick(P.gap_kmin, P.gap_n, P.gap_thr, c.x);
                sr = span_pick(P.size_kmin, P.size_n, P.size_thr, c.y);
            }
            const bool act = lane < np;
            const uint32_t p = p0 + (uint32_t)lane;
            // saturate so the prefix sums cannot wrap (any value >= n ends the row)
            const uint32_t gs = !act ? 0u : gr > (uint32_t)n ? (uint32_t)n : gr;
            const uint32_t ss_ = !act ? 0u : sr > (uint32_t)n ? (uint32_t)n : sr;
            const uint32_t step = gs + ss_;
            const uint32_t incl = wave_incl_sum(step), incl_s = wave_incl_sum(ss_);
            const int Ip = I0 + (int)(incl - step);            // id cursor at the start of pass p
            const int Ap = A0 + (int)(incl_s - ss_);           // ids spanned before p
            const bool last = act && Ip + (int)step >= n && Ip < n;  // the pass where ip reaches n
            const uint64_t lm = __ballot(last);
            const int Pl = lm ? __builtin_ctzll(lm) : 64;     // lane of the last pass (64: none this round)
            const int nr = Pl < 64 ? Pl + 1 : np;             // passes written this round
            const int lp = Ip - Ap + (int)p;                   // input cursor
            const int ap = Ap + (int)p;                        // label cursor
            const int gg = lane == Pl ? ((int)gs < n - Ip ? (int)gs : n - Ip) : (int)gs;
            const int ip1 = Ip + gg;
            const int sz = lane == Pl ? ((int)ss_ < n - ip1 ? (int)ss_ : n - ip1) : (int)ss_;
            if (lane < nr) {
                sp[lane] = SpanPass{(uint32_t)lp | (uint32_t)gg << 16, (uint32_t)Ip | (uint32_t)sz << 16, (uint32_t)ap, p};
                // the reference's panics, counted: a sentinel index >= 100, label writes past S/4
                if (sz > 0) {
                    bad += p >= 100u ? 1u : 0u;
                    const int lo = ap > LW ? ap : LW, hi = ap + sz + 1;
                    bad += hi > lo ? (uint32_t)(hi - lo) : 0u;
                }
                if (lane == Pl) {
                    bad += p + 1u >= 100u ? 1u : 0u;
                    bad += ap + (sz > 0 ? sz + 1 : 0) >= LW ? 1u : 0u;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            // ---- B. this round's positions ----
            const int lpA = lane_bcast(lp, 0);
            const int lpB = lane_bcast(lp + gg + (sz > 0 ? 1 : 0), nr - 1);
            const int apA = lane_bcast(ap, 0);
            const int apB = lane_bcast(ap + (sz > 0 ? sz + 1 : 0), nr - 1);
            int own = 0;  // pass of the group's first position (wave-uniform)
            for (int b = lpA; b < lpB; b += 64) {
                const int q = b + lane;
                int o = own;
                for (int t = own + 1; t < nr; ++t) {
                    const int st = lane_bcast(lp, t);
                    if (st >= b + 64) break;
                    o = q >= st ? t : o;
                }
                own = lane_bcast(o, 63);
                if (q < lpB) {
                    const SpanPass e = sp[o];
                    const int off = q - (int)(e.lp_gg & 0xFFFFu);
                    const int ge = (int)(e.lp_gg >> 16);
                    st_nt(ids_o + q, off < ge ? rid[(int)(e.ip_sz & 0xFFFFu) + off] : extra(e.pass));
                }
            }
            own = 0;
            const int apLim = apB < LW ? apB : LW;
            for (int b = apA; b < apLim; b += 64) {
                const int q = b + lane;
                int o = own;
                for (int t = own + 1; t < nr; ++t) {
                    const int st = lane_bcast(ap, t);
                    if (st >= b + 64) break;
                    o = q >= st ? t : o;
                }
                own = lane_bcast(o, 63);
                if (q < apLim) {
                    const SpanPass e = sp[o];
                    const int off = q - (int)e.ap;
                    st_nt(lb_o + q, off == 0 ? extra(e.pass)
                                            : rid[(int)(e.ip_sz & 0xFFFFu) + (int)(e.lp_gg >> 16) + off - 1]);
                }
            }
            if (Pl < 64) {
                lp_end = lpB;
                ap_end = apB;
                if (lane == 0 && ap_end < LW) st_nt(lb_o + ap_end, extra((uint32_t)lane_bcast((int)p, Pl) + 1u));
                break;
            }
            I0 += (int)lane_bcast((int)incl, 63);
            A0 += (int)lane_bcast((int)incl_s, 63);
            p0 += (uint32_t)np;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
        for (int j = lp_end + lane; j < S; j += 64) st_nt(ids_o + j, 0);
        for (int j = ap_end + 1 + lane; j < LW; j += 64) st_nt(lb_o + j, -100);
        for (int d = 32; d >= 1; d >>= 1) bad += __shfl_xor(bad, d, 64);
        if (lane == 0 && bad) atomicAdd(err, bad);
    }
}

// ---------------------------------------------------------------------------
// Span rows in two phases.
//  1. k_span_plan, one lane per row: the row's passes drawn and walked
//     serially (the cursor recurrence above, lane-local), each pass written to
//     the row's plan as {lp | gg << 16, ip | sz << 16}; the row's pass count
//     and its ids / labels ends to meta.  A row whose passes overrun the plan
//     (capr = LW / 2 + 2: every row within the label width fits, so only rows
//     the reference panics on can) is listed for the one-pass kernel instead.
//  2. k_span_write, one wave per row: framed ids and plan in LDS, the pass
//     starts scattered into per-position marks, a max-scan gives every
//     position its pass, and each lane writes 4 contiguous positions per
//     store -- the row writer of k_rows, no serial walk.
// ---------------------------------------------------------------------------
struct LaneStream {  // rng_mode 1: one lane's StdRng stream, its current ChaCha12 block in LDS
    uint32_t key[8];
    uint32_t *blk;  // 16 words (LDS, this lane's)
    int64_t have;
    __device__ uint64_t at(uint64_t k) {
        const int64_t b = (int64_t)(k >> 3);
        if (b != have) {
            uint32_t o[16];
            chacha12_block(key, (uint32_t)b, o);
#pragma unroll
            for (int q = 0; q < 16; ++q) blk[q] = o[q];
            have = b;
        }
        const uint32_t w = 2u * (uint32_t)(k & 7u);
        return (uint64_t)blk[w + 1] << 32 | blk[w];
    }
};

template <int RAND>
__global__ __launch_bounds__(256) void k_span_plan(RowParams P, const uint32_t *__restrict__ rec_cnt,
                                                   const uint32_t *__restrict__ row_off,
                                                   const uint32_t *__restrict__ row_rec, SegSel sel, int64_t rows_cap,
                                                   SpanPlan pl, uint32_t *__restrict__ err) {
    __shared__ uint32_t s_blk[RAND ? 256 : 1][17];
    const int S = P.S, LW = P.label_width;
    const RowSpan rs = row_span(sel, row_off, P.B, rows_cap);
    uint32_t bad = 0;
    for (int64_t g = rs.g_lo + (int64_t)blockIdx.x * 256 + threadIdx.x; g < rs.g_real;
         g += (int64_t)gridDim.x * 256) {
        const int64_t r = row_rec[g];
        const uint32_t k = (uint32_t)(g - row_off[r]);
        const int64_t nf = (int64_t)rec_cnt[r] + P.n_pre + P.n_post;
        const int64_t base = P.chunk ? (int64_t)k * S : 0;
        const int n = (int)((nf - base) < S ? (nf - base) : S);
        if (n <= 0) {
            pl.meta[g] = make_uint2(0u, 0u);
            continue;
        }
        const uint64_t rec = P.first_record + (uint64_t)r;
        LaneStream ls;
        uint64_t spos = 0;
        if (RAND) {
            const uint32_t kk[8] = {(uint32_t)P.seed, (uint32_t)(P.seed >> 32), (uint32_t)rec, (uint32_t)(rec >> 32),
                                    k, 0u, 0u, 0u};
#pragma unroll
            for (int q = 0; q < 8; ++q) ls.key[q] = kk[q];
            ls.blk = s_blk[RAND ? threadIdx.x : 0];
            ls.have = -1;
        }
        uint2 *tab = pl.tab + g * (int64_t)pl.capr;
        uint32_t rbad = 0;
        int Ip = 0, Ap = 0;
        bool over = false;
        for (uint32_t p = 0;; ++p) {
            uint32_t gr, sr;
            if (RAND) {
                uint32_t l1, l2;
                const double d1 = zig_normal(ls, spos, P.zig_x, P.zig_f, &l1);
                const double d2 = zig_normal(ls, spos + l1, P.zig_x, P.zig_f, &l2);
                spos += l1 + l2;
                gr = sat_draw(P.avg_span_gap - d1, n);
                const uint32_t sz = sat_draw(P.avg_span_size - d2, n);
                sr = sz > 1u ? sz : 1u;  // std::cmp::max(distance as usize, 1)
            } else {
                const uint4 c = philox4x32_10(make_uint4(p, k | 0x40000000u, (uint32_t)rec, (uint32_t)(rec >> 32)),
                                              (uint32_t)P.seed, (uint32_t)(P.seed >> 32));
                gr = span_pick(P.gap_kmin, P.gap_n, P.gap_thr, c.x);
                sr = span_pick(P.size_kmin, P.size_n, P.size_thr, c.y);
            }
            const int gs = gr > (uint32_t)n ? n : (int)gr, ss = sr > (uint32_t)n ? n : (int)sr;
            const bool last = Ip + gs + ss >= n;
            const int gg = last ? (gs < n - Ip ? gs : n - Ip) : gs;
            const int sz = last ? (ss < n - Ip - gg ? ss : n - Ip - gg) : ss;
            const int lp = Ip - Ap + (int)p, ap = Ap + (int)p;
            if ((int)p >= pl.capr) {
                over = true;
                break;
            }
            tab[p] = make_uint2((uint32_t)lp | (uint32_t)gg << 16, (uint32_t)Ip | (uint32_t)sz << 16);
            // the reference's panics, counted as k_rows_span counts them
            if (sz > 0) {
                rbad += p >= 100u ? 1u : 0u;
                const int lo = ap > LW ? ap : LW, hi = ap + sz + 1;
                rbad += hi > lo ? (uint32_t)(hi - lo) : 0u;
            }
            if (last) {
                rbad += p + 1u >= 100u ? 1u : 0u;
                rbad += ap + (sz > 0 ? sz + 1 : 0) >= LW ? 1u : 0u;
                const uint32_t lp_end = (uint32_t)(lp + gg + (sz > 0 ? 1 : 0));
                const uint32_t ap_end = (uint32_t)(ap + (sz > 0 ? sz + 1 : 0));
                pl.meta[g] = make_uint2(p + 1u, lp_end | ap_end << 16);
                break;
            }
            Ip += gs + ss;
            Ap += ss;
        }
        if (over) {  // the one-pass kernel takes this row (and counts its errors)
            pl.meta[g] = make_uint2(0xFFFFFFFFu, 0u);
            pl.ovf_list[atomicAdd(pl.ovf_n, 1u)] = (uint32_t)g;
        } else {
            bad += rbad;
        }
    }
    for (int d = 32; d >= 1; d >>= 1) bad += __shfl_xor(bad, d, 64);
    if ((threadIdx.x & 63) == 0 && bad) atomicAdd(err, bad);
}

#define MAX_U32(a, b) ((a) > (b) ? (a) : (b))
// Positions [0, W) of one plane of a row, lane L holding 256 m + 4 L + w: the
// owner pass of each position = the max-scan of `mk` (pass p marked at its
// first position); val(q, owner) gives the value; positions >= end get
// tail(q).  Stores of 16 B per lane when W is a multiple of 4.
template <class Val, class Tail>
__device__ __forceinline__ void span_plane(int32_t *__restrict__ o, int W, int end, const uint16_t *mk, Val val,
                                           Tail tail) {
    const int lane = lane_id();
    uint32_t carry = 0;
    const bool vec = (W & 3) == 0;
    for (int b = 0; b < W; b += 256) {
        const int q0 = b + 4 * lane;
        uint32_t own[4], run = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int q = q0 + w;
            const uint32_t m = q < end ? (uint32_t)mk[q] : 0u;
            run = MAX_U32(run, m);
            own[w] = run;
        }
        uint32_t x = run;
        DPP_SCAN(x, MAX_U32);
        // (the DPP read once, unconditionally: inside the macro's ternary it was evaluated
        // twice and the compiler made the second a branch -- a cross-lane read under a
        // partial exec mask, which reads 0 from the inactive neighbours)
        const uint32_t prev = wave_prev(x), last = (uint32_t)lane_bcast((int)x, 63);
        const uint32_t before = prev > carry ? prev : carry;
        carry = carry > last ? carry : last;
        int32_t v[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int q = q0 + w;
            v[w] = q < end ? val(q, MAX_U32(own[w], before)) : tail(q);
        }
        if (vec) {
            typedef int32_t v4i __attribute__((ext_vector_type(4)));
            if (q0 < W) __builtin_nontemporal_store(v4i{v[0], v[1], v[2], v[3]}, reinterpret_cast<v4i *>(o + q0));
        } else {
#pragma unroll
            for (int w = 0; w < 4; ++w)
                if (q0 + w < W) st_nt(o + q0 + w, v[w]);
        }
    }
}

constexpr int SPAN_TABL = 128;  // plan entries per row held in LDS (the rest read from the plan)

__global__ __launch_bounds__(256) void k_span_write(RowParams P, const uint32_t *__restrict__ tok,
                                                    const uint32_t *__restrict__ rec_tok,
                                                    const uint32_t *__restrict__ rec_cnt,
                                                    const uint32_t *__restrict__ row_off,
                                                    const uint32_t *__restrict__ row_rec, SegSel sel,
                                                    int64_t rows_cap, RowOut out, SpanPlan pl) {
    __shared__ int32_t s_extra[100];
    __shared__ uint2 s_tab[4][SPAN_TABL > 0 ? SPAN_TABL : 1];
    extern __shared__ int32_t s_dyn[];  // per wave: rid[S] | mk[S] u16 | mk2[LW] u16 (rounded)
    const int lane = lane_id();
    const int wid = (int)(threadIdx.x >> 6);
    if (threadIdx.x < 100) s_extra[threadIdx.x] = P.extra_ids[threadIdx.x];
    __syncthreads();
    const int S = P.S, LW = P.label_width;
    const int wave_words = S + ((S + LW + 1) >> 1);
    int32_t *rid = s_dyn + (size_t)wid * wave_words;
    uint16_t *mk = reinterpret_cast<uint16_t *>(rid + S);
    uint16_t *mk2 = mk + S;
    uint2 *tl = s_tab[wid];
    const RowSpan rs = row_span(sel, row_off, P.B, rows_cap);
    const int64_t G = rs.g_real;
    auto extra = [&](uint32_t q) -> int32_t { return s_extra[q < 100u ? q : 99u]; };
    auto fence = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
    for (int64_t g = rs.g_lo + (int64_t)blockIdx.x * 4 + wid; g < rs.g_end; g += (int64_t)gridDim.x * 4) {
        int32_t *ids_o = out.input_ids + g * S;
        int32_t *am_o = out.attention_mask + g * S;
        int32_t *lb_o = out.labels + g * (int64_t)LW;
        const uint2 m = g < G ? pl.meta[g] : make_uint2(0u, 0u);
        if (m.x == 0xFFFFFFFFu) continue;  // the one-pass kernel's row
        for (int j = lane; j < S; j += 64) st_nt(am_o + j, 1);  // attention stays 1 (the zeroing loop is empty)
        const int np = (int)m.x;
        if (np == 0) {  // past the last row (or an empty one): T5Data::new's values
            for (int j = lane; j < S; j += 64) st_nt(ids_o + j, 0);
            for (int j = lane; j < LW; j += 64) st_nt(lb_o + j, -100);
            continue;
        }
        const int lp_end = (int)(m.y & 0xFFFFu), ap_end = (int)(m.y >> 16);
        const int64_t r = row_rec[g];
        const uint32_t k = (uint32_t)(g - row_off[r]);
        const uint32_t cnt = rec_cnt[r];
        const uint32_t t0 = rec_tok[r];
        const int64_t nf = (int64_t)cnt + P.n_pre + P.n_post;
        const int64_t base = P.chunk ? (int64_t)k * S : 0;
        const int n = (int)((nf - base) < S ? (nf - base) : S);
        const uint2 *tab = pl.tab + g * (int64_t)pl.capr;
        auto fid = [&](int j) -> int32_t {  // framed id j of this chunk
            const int64_t f = base + j;
            if (f < P.n_pre) return frame_id(P.pre, (int)f);
            if (f < P.n_pre + (int64_t)cnt) return (int32_t)tok[t0 + (f - P.n_pre)];
            return frame_id(P.post, (int)(f - P.n_pre - cnt));
        };
        // framed ids, plan and zeroed marks into LDS: every load in flight together
        for (int j0 = 0; j0 < n; j0 += 64 * 8) {
            int32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int j = j0 + 64 * u + lane;
                v[u] = j < n ? fid(j) : 0;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int j = j0 + 64 * u + lane;
                if (j < n) rid[j] = v[u];
            }
        }
        for (int p = lane; p < np && p < SPAN_TABL; p += 64) tl[p] = tab[p];
        for (int j = 2 * lane; j < S + LW; j += 128) *reinterpret_cast<uint32_t *>(mk + j) = 0u;
        fence();
        auto ent = [&](int p) -> uint2 { return p < SPAN_TABL ? tl[p] : tab[p]; };
        // pass starts: ids at lp, labels at ap = ip - lp + 2 p (within the label width)
        for (int p = lane; p < np; p += 64) {
            const uint2 e = ent(p);
            const int lp = (int)(e.x & 0xFFFFu), ip = (int)(e.y & 0xFFFFu);
            const int ap = ip - lp + 2 * p;
            if (lp < S) mk[lp] = (uint16_t)p;
            if (ap < LW) mk2[ap] = (uint16_t)p;
        }
        fence();
        span_plane(
            ids_o, S, lp_end, mk,
            [&](int q, uint32_t o) -> int32_t {
                const uint2 e = ent((int)o);
                const int off = q - (int)(e.x & 0xFFFFu), ge = (int)(e.x >> 16);
                return off < ge ? rid[(int)(e.y & 0xFFFFu) + off] : extra(o);
            },
            [&](int) -> int32_t { return 0; });
        const int apLim = ap_end < LW ? ap_end : LW;
        const int32_t fin = extra((uint32_t)np);  // <extra_id_{last pass + 1}>
        span_plane(
            lb_o, LW, apLim, mk2,
            [&](int q, uint32_t o) -> int32_t {
                const uint2 e = ent((int)o);
                const int lp = (int)(e.x & 0xFFFFu), ge = (int)(e.x >> 16), ip = (int)(e.y & 0xFFFFu);
                const int off = q - (ip - lp + 2 * (int)o);
                return off == 0 ? extra(o) : rid[ip + ge + off - 1];
            },
            [&](int q) -> int32_t { return q == ap_end ? fin : -100; });
        fence();  // (the next row rewrites rid / marks)
    }
}

hipError_t launch_rows_span(const RowParams &P, const uint32_t *tok, const uint32_t *rec_tok, const uint32_t *rec_cnt,
                            const uint32_t *row_off, const uint32_t *row_rec, SegSel sel, int64_t rows_cap,
                            RowOut out, uint32_t *err, hipStream_t st, const SpanPlan *pl) {
    if (rows_cap == 0) return hipSuccess;
    if (P.S > 65535 || (P.rng_mode == 1 && (!P.zig_x || !P.zig_f))) return hipErrorInvalidValue;
    if (sel.k == 0) {  // the error count covers the whole call
        hipError_t e = hipMemsetAsync(err, 0, sizeof(uint32_t), st);
        if (e != hipSuccess) return e;
    }
    if (pl) {
        if (P.S > 16384 || pl->capr < 1) return hipErrorInvalidValue;
        hipError_t e = hipMemsetAsync(pl->ovf_n, 0, sizeof(uint32_t), st);
        if (e != hipSuccess) return e;
        const int64_t pb = (rows_cap + 255) / 256;
        const unsigned pgrid = (unsigned)(pb < 8192 ? pb : 8192);
        if (P.rng_mode == 1)
            hipLaunchKernelGGL(k_span_plan<1>, dim3(pgrid), dim3(256), 0, st, P, rec_cnt, row_off, row_rec, sel,
                               rows_cap, *pl, err);
        else
            hipLaunchKernelGGL(k_span_plan<0>, dim3(pgrid), dim3(256), 0, st, P, rec_cnt, row_off, row_rec, sel,
                               rows_cap, *pl, err);
        const int64_t want = (rows_cap + 3) / 4;
        const unsigned grid = (unsigned)(want < SPAN_GRID_CAP ? want : SPAN_GRID_CAP);
        const size_t dyn = (size_t)4 * 4 * (P.S + ((P.S + P.label_width + 1) >> 1));
        hipLaunchKernelGGL(k_span_write, dim3(grid), dim3(256), dyn, st, P, tok, rec_tok, rec_cnt, row_off, row_rec,
                           sel, rows_cap, out, *pl);
        // rows whose passes overran the plan: the one-pass kernel over the list
        const size_t dyn1 = (size_t)4 * P.S * sizeof(int32_t);
        const unsigned lgrid = 256;
        if (P.rng_mode == 1)
            hipLaunchKernelGGL(k_rows_span<1>, dim3(lgrid), dim3(256), dyn1, st, P, tok, rec_tok, rec_cnt, row_off,
                               row_rec, sel, rows_cap, out, err, pl->ovf_list, pl->ovf_n);
        else
            hipLaunchKernelGGL(k_rows_span<0>, dim3(lgrid), dim3(256), dyn1, st, P, tok, rec_tok, rec_cnt, row_off,
                               row_rec, sel, rows_cap, out, err, pl->ovf_list, pl->ovf_n);
        return hipGetLastError();
    }
    const int64_t want = (rows_cap + 3) / 4;
    const unsigned grid = (unsigned)(want < SPAN_GRID_CAP ? want : SPAN_GRID_CAP);
    const size_t dyn = (size_t)4 * P.S * sizeof(int32_t);  // s_rid
    if (P.rng_mode == 1)
        hipLaunchKernelGGL(k_rows_span<1>, dim3(grid), dim3(256), dyn, st, P, tok, rec_tok, rec_cnt, row_off, row_rec,
                           sel, rows_cap, out, err, nullptr, nullptr);
    else
        hipLaunchKernelGGL(k_rows_span<0>, dim3(grid), dim3(256), dyn, st, P, tok, rec_tok, rec_cnt, row_off, row_rec,
                           sel, rows_cap, out, err, nullptr, nullptr);
    return hipGetLastError();
}

// BertData MultiLabel branch (bert_data.rs:66-78): labels_f32[row] = zeros with
// 1.0 at each Label::Multi index.  An index >= number_labels (the reference
// panics) is skipped and counted in *err.  Rows past the last batch: zeros.
__global__ __launch_bounds__(256) void k_multi_labels(const uint32_t *__restrict__ labels,
                                                      const uint64_t *__restrict__ label_off,
                                                      const uint32_t *__restrict__ row_rec,
                                                      const uint32_t *__restrict__ row_off, SegSel sel,
                                                      int64_t rows_cap, int B, int NL, float *__restrict__ out,
                                                      uint32_t *__restrict__ err) {
    const RowSpan rs = row_span(sel, row_off, B, rows_cap);
    const int64_t G = rs.g_real;
    for (int64_t g = rs.g_lo + (int64_t)blockIdx.x * 256 + threadIdx.x; g < rs.g_end; g += (int64_t)gridDim.x * 256) {
        float *o = out + g * NL;
        for (int k = 0; k < NL; ++k) o[k] = 0.f;
        if (g >= (int64_t)G || !labels) continue;
        const uint32_t r = row_rec[g];
        uint32_t bad = 0;
        for (uint64_t i = label_off[r]; i < label_off[r + 1]; ++i) {
            const uint32_t x = labels[i];
            if (x < (uint32_t)NL) o[x] = 1.f;
            else ++bad;
        }
        if (bad) atomicAdd(err, bad);
    }
}

hipError_t launch_multi_labels(const uint32_t *labels, const uint64_t *label_off, const uint32_t *row_rec,
                               const uint32_t *row_off, SegSel sel, int64_t rows_cap, int B, int NL, float *out,
                               uint32_t *err, hipStream_t st) {
    if (rows_cap == 0) return hipSuccess;
    const int64_t want = (rows_cap + 255) / 256;
    hipLaunchKernelGGL(k_multi_labels, dim3((unsigned)(want < 2048 ? want : 2048)), dim3(256), 0, st, labels,
                       label_off, row_rec, row_off, sel, rows_cap, B, NL, out, err);
    return hipGetLastError();
}

// BertData SingleClass branch (bert_data.rs:79-81: label.map(|s| self.label.push(s))),
// fed by SingleClassArrowGenerator (single_arrow.rs:16-26), which always yields
// Some(Label::Single): labels[row] = the record's one label.  A record with a
// label count other than one is counted in *err (label 0 written).  Rows past the
// last batch: 0 (BertData's label list has one entry per filled row).
__global__ __launch_bounds__(256) void k_single_labels(const uint32_t *__restrict__ labels,
                                                       const uint64_t *__restrict__ label_off,
                                                       const uint32_t *__restrict__ row_rec,
                                                       const uint32_t *__restrict__ row_off, SegSel sel,
                                                       int64_t rows_cap, int B, int32_t *__restrict__ out,
                                                       uint32_t *__restrict__ err) {
    const RowSpan rs = row_span(sel, row_off, B, rows_cap);
    const int64_t G = rs.g_real;
    for (int64_t g = rs.g_lo + (int64_t)blockIdx.x * 256 + threadIdx.x; g < rs.g_end; g += (int64_t)gridDim.x * 256) {
        int32_t v = 0;
        if (g < (int64_t)G && labels) {
            const uint32_t r = row_rec[g];
            const uint64_t a = label_off[r], e = label_off[r + 1];
            if (e == a + 1) v = (int32_t)labels[a];
            else atomicAdd(err, 1u);
        }
        out[g] = v;
    }
}

hipError_t launch_single_labels(const uint32_t *labels, const uint64_t *label_off, const uint32_t *row_rec,
                                const uint32_t *row_off, SegSel sel, int64_t rows_cap, int B, int32_t *out,
                                uint32_t *err, hipStream_t st) {
    if (rows_cap == 0) return hipSuccess;
    const int64_t want = (rows_cap + 255) / 256;
    hipLaunchKernelGGL(k_single_labels, dim3((unsigned)(want < 2048 ? want : 2048)), dim3(256), 0, st, labels,
                       label_off, row_rec, row_off, sel, rows_cap, B, out, err);
    return hipGetLastError();
}

}  // namespace sdl
