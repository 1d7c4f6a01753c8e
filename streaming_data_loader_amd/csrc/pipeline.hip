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

__global__ __launch_bounds__(SCAN_NT) void k_scan_sums(uint32_t *__restrict__ sums, int64_t nb) {
    __shared__ uint32_t scratch[SCAN_NT / 64];
    uint32_t carry = 0;
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

int64_t scan_tmp_words(int64_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE + 1; }

hipError_t launch_exclusive_scan(const uint32_t *in, uint32_t *out, int64_t n, uint32_t *tmp, hipStream_t st) {
    if (n <= 0) return hipMemsetAsync(out, 0, sizeof(uint32_t), st);
    const int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)nb), dim3(SCAN_NT), 0, st, in, n, tmp);
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(SCAN_NT), 0, st, tmp, nb);
    hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)nb), dim3(SCAN_NT), 0, st, in, n, tmp, nb, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Per-chunk token lists -> one dense token array in arena order.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_compact_tokens(const uint32_t *__restrict__ tokc,
                                                        const uint32_t *__restrict__ chunk_cnt,
                                                        const uint32_t *__restrict__ chunk_off,
                                                        uint32_t *__restrict__ tok) {
    const uint32_t n = chunk_cnt[blockIdx.x];
    const uint32_t *src = tokc + (int64_t)blockIdx.x * STAGE;
    uint32_t *dst = tok + chunk_off[blockIdx.x];
    for (uint32_t i = threadIdx.x; i < n; i += 256) dst[i] = src[i];
}

hipError_t launch_compact_tokens(const uint32_t *tokc, const uint32_t *chunk_cnt, const uint32_t *chunk_off,
                                 int64_t n_chunks, uint32_t *tok, hipStream_t st) {
    if (n_chunks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_compact_tokens, dim3((unsigned)n_chunks), dim3(256), 0, st, tokc, chunk_cnt, chunk_off, tok);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Per record: where its ids start, how many, and how many rows it yields.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_records(RowParams P, const uint64_t *__restrict__ off, int64_t R, int64_t N,
                                                 const uint32_t *__restrict__ chunk_off, int64_t n_chunks,
                                                 const uint32_t *__restrict__ rec_local, uint32_t *__restrict__ rec_tok,
                                                 uint32_t *__restrict__ rec_cnt, uint32_t *__restrict__ rec_rows) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= R) return;
    const uint32_t total = chunk_off[n_chunks];
    auto tok_off = [&](int64_t q) -> uint32_t {
        const int64_t p = (int64_t)off[q];
        return p >= N ? total : chunk_off[p / CHUNK] + rec_local[q];
    };
    const uint32_t a = tok_off(r), b = tok_off(r + 1);
    const uint32_t cnt = b - a;
    const uint32_t n = cnt + (uint32_t)(P.n_pre + P.n_post);  // encode_mask framing
    uint32_t rows = 0;
    if (n >= (uint32_t)P.min_ids) rows = P.chunk ? ceil_div_u32(n, (uint32_t)P.S) : 1u;  // gen_batcher.rs:74-80
    rec_tok[r] = a;
    rec_cnt[r] = cnt;
    rec_rows[r] = rows;
}

hipError_t launch_records(const RowParams &P, const uint64_t *off, int64_t R, int64_t N, const uint32_t *chunk_off,
                          int64_t n_chunks, const uint32_t *rec_local, uint32_t *rec_tok, uint32_t *rec_cnt,
                          uint32_t *rec_rows, hipStream_t st) {
    if (R == 0) return hipSuccess;
    hipLaunchKernelGGL(k_records, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, st, P, off, R, N, chunk_off,
                       n_chunks, rec_local, rec_tok, rec_cnt, rec_rows);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// RNG contract: Philox4x32-10 (Salmon et al., SC'11), as oracle/sdl_oracle.c.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
        const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
        c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

__device__ __forceinline__ uint32_t mlm_key(uint64_t seed, uint64_t rec, uint32_t chunk, uint32_t pos) {
    const uint4 c = philox4x32_10(make_uint4(pos >> 2, chunk, (uint32_t)rec, (uint32_t)(rec >> 32)), (uint32_t)seed,
                                  (uint32_t)(seed >> 32));
    const uint32_t s = pos & 3u;
    return s == 0 ? c.x : s == 1 ? c.y : s == 2 ? c.z : c.w;
}

// Marks the k smallest (key, position) pairs of a row held as key[m] at
// position lane + 64*m.  32-step radix select of the k-th smallest key with
// wave ballots, then position-ordered tie-break among equal keys.
template <int M>
__device__ __forceinline__ void select_k_smallest(const uint32_t (&key)[M], int k, bool (&sel)[M]) {
    if (k <= 0) {
#pragma unroll
        for (int m = 0; m < M; ++m) sel[m] = false;
        return;
    }
    uint32_t prefix = 0;
    for (int bit = 31; bit >= 0; --bit) {
        const uint32_t cand = prefix | (1u << bit);
        int c = 0;
#pragma unroll
        for (int m = 0; m < M; ++m) c += __popcll(__ballot(key[m] < cand));
        if (c < k) prefix = cand;
    }
    int c_lt = 0;
#pragma unroll
    for (int m = 0; m < M; ++m) c_lt += __popcll(__ballot(key[m] < prefix));
    const int need = k - c_lt;
    const uint64_t lt_mask = (1ull << lane_id()) - 1ull;
    int before = 0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
        const uint64_t eq = __ballot(key[m] == prefix);
        const int rank = before + __popcll(eq & lt_mask);
        sel[m] = key[m] < prefix || (key[m] == prefix && rank < need);
        before += __popcll(eq);
    }
}

template <int M>
__global__ __launch_bounds__(256) void k_rows(RowParams P, const uint32_t *__restrict__ tok,
                                              const uint32_t *__restrict__ rec_tok, const uint32_t *__restrict__ rec_cnt,
                                              const uint32_t *__restrict__ row_off, int64_t R,
                                              const uint32_t *__restrict__ d_rows, int64_t rows_cap, RowOut out) {
    const int lane = lane_id();
    const int wid = (int)(threadIdx.x >> 6);
    const int S = P.S;
    const uint32_t G = *d_rows;
    int64_t Gpad = ((int64_t)G + P.B - 1) / P.B * P.B;
    if (Gpad > rows_cap) Gpad = rows_cap;
    for (int64_t g = (int64_t)blockIdx.x * 4 + wid; g < Gpad; g += (int64_t)gridDim.x * 4) {
        int32_t *ids_o = out.input_ids + g * S;
        int32_t *am_o = out.attention_mask + g * S;
        int32_t *tt_o = out.token_type_ids ? out.token_type_ids + g * S : nullptr;
        int32_t *lb_o = out.labels + g * (int64_t)P.label_width;
        if (g >= (int64_t)G) {  // rows of the last batch nobody filled: initial values
#pragma unroll
            for (int m = 0; m < M; ++m) {
                const int j = lane + 64 * m;
                if (j < S) {
                    ids_o[j] = 0;
                    am_o[j] = 1;
                    if (tt_o) tt_o[j] = 0;
                }
                if (j < P.label_width) lb_o[j] = -100;
            }
            continue;
        }
        // record of row g: last r with row_off[r] <= g
        int64_t lo = 0, hi = R;
        while (hi - lo > 1) {
            const int64_t mid = (lo + hi) >> 1;
            if ((int64_t)row_off[mid] <= g) lo = mid; else hi = mid;
        }
        const int64_t r = lo;
        const uint32_t k = (uint32_t)(g - row_off[r]);
        const uint32_t cnt = rec_cnt[r];
        const uint32_t t0 = rec_tok[r];
        const int64_t n = (int64_t)cnt + P.n_pre + P.n_post;
        const int64_t base = P.chunk ? (int64_t)k * S : 0;
        const int l = (int)((n - base) < S ? (n - base) : S);

        int32_t id[M];
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const int j = lane + 64 * m;
            int32_t v = 0;
            if (j < l) {
                const int64_t f = base + j;
                if (f < P.n_pre) v = P.pre[f];
                else if (f < P.n_pre + (int64_t)cnt) v = (int32_t)tok[t0 + (f - P.n_pre)];
                else v = P.post[f - P.n_pre - cnt];
            }
            id[m] = v;
        }
        const uint64_t rec = P.first_record + (uint64_t)r;
        if (P.task == 0) {  // MLM: BertData::mask_batch
            uint32_t key[M];
#pragma unroll
            for (int m = 0; m < M; ++m) {
                const int j = lane + 64 * m;
                key[m] = j < S ? mlm_key(P.seed, rec, k, (uint32_t)j) : 0xFFFFFFFFu;
            }
            bool sel[M];
            select_k_smallest<M>(key, P.mask_length, sel);
#pragma unroll
            for (int m = 0; m < M; ++m) {
                const int j = lane + 64 * m;
                if (j >= S) continue;
                int32_t lab = -100, v = id[m];
                if (sel[m] && v != 0) {
                    lab = v;
                    v = P.mask_id;
                }
                ids_o[j] = v;
                am_o[j] = (l < S && j >= S - l) ? 0 : 1;  // reversed-range quirk (bert_data.rs:58-63)
                if (tt_o) tt_o[j] = 0;
                lb_o[j] = lab;
            }
        } else {  // CLM: GptData::put_data, labels = row as i32 (no shift)
#pragma unroll
            for (int m = 0; m < M; ++m) {
                const int j = lane + 64 * m;
                if (j >= S) continue;
                const bool tail = l < S && j >= S - l;  // gpt_data.rs:33-41
                ids_o[j] = id[m];
                am_o[j] = tail ? 0 : 1;
                lb_o[j] = tail ? -100 : id[m];
                if (tt_o) tt_o[j] = 0;
            }
        }
    }
}

hipError_t launch_rows(const RowParams &P, const uint32_t *tok, const uint32_t *rec_tok, const uint32_t *rec_cnt,
                       const uint32_t *row_off, int64_t R, const uint32_t *d_rows, int64_t rows_cap, RowOut out,
                       hipStream_t st) {
    if (rows_cap == 0) return hipSuccess;
    const int64_t want = (rows_cap + 3) / 4;
    const unsigned grid = (unsigned)(want < 4096 ? want : 4096);
    const int M = (P.S + 63) / 64;
#define SDL_ROWS(MM)                                                                                                 \
    hipLaunchKernelGGL(k_rows<MM>, dim3(grid), dim3(256), 0, st, P, tok, rec_tok, rec_cnt, row_off, R, d_rows, \
                       rows_cap, out)
    if (M <= 1) SDL_ROWS(1);
    else if (M <= 2) SDL_ROWS(2);
    else if (M <= 4) SDL_ROWS(4);
    else if (M <= 8) SDL_ROWS(8);
    else if (M <= 16) SDL_ROWS(16);
    else if (M <= 32) SDL_ROWS(32);
    else return hipErrorInvalidValue;
#undef SDL_ROWS
    return hipGetLastError();
}

}  // namespace sdl
