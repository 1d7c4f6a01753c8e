// Device code shared by the rows kernels (pipeline.hip) and the fused tiny-push tail of the
// WordPiece chunk kernel (tokenize_wordpiece.hip): chunk-list compaction, per-record framing,
// the Philox mask contract and one row's planes.
#pragma once
#include "common.hpp"
#include "device_util.hpp"
#include "kernels.hpp"

namespace sdl {

constexpr int COMPACT_CPW = 4;  // chunks per wave: their loads are in flight together
// one wave: chunks [cb, cb + COMPACT_CPW).  PART 1: only when the call has no long items, 2: only
// when it has (separate kernels keep the plain copy's registers), 0: either.
template <int PART = 0>
__device__ __forceinline__ void compact_wave(int64_t cb, const uint32_t *__restrict__ tokc,
                                             const uint32_t *__restrict__ chunk_cnt,
                                             const uint32_t *__restrict__ chunk_off, int64_t n_chunks,
                                             uint32_t *__restrict__ tok, const uint32_t *long_count,
                                             const uint32_t *__restrict__ chunk_ent,
                                             const BpeLong *__restrict__ long_list,
                                             const uint16_t *__restrict__ long_scratch,
                                             const uint32_t *__restrict__ long_pool, int64_t stride) {
    const int lane = threadIdx.x & 63;
    uint32_t n[COMPACT_CPW], o[COMPACT_CPW];
#pragma unroll
    for (int j = 0; j < COMPACT_CPW; ++j) {
        const bool in = cb + j < n_chunks;
        n[j] = in ? chunk_cnt[cb + j] : 0u;
        o[j] = in ? chunk_off[cb + j] : 0u;
    }
    // (unigram: Viterbi job markers are in every call's lists)
    const bool has_long = long_count && (long_pool != nullptr || *long_count != 0);
    if ((PART == 1 && has_long) || (PART == 2 && !has_long)) return;
    if (!has_long) {
        // lane-contiguous dwords: every store instruction writes 256 B of the
        // dense array back to back (at any alignment); the first 256 ids of all
        // the wave's chunks are loaded before any is stored
        uint32_t v[COMPACT_CPW][4];
#pragma unroll
        for (int j = 0; j < COMPACT_CPW; ++j)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t i = 64 * k + lane;
                v[j][k] = i < n[j] ? __builtin_nontemporal_load(tokc + (cb + j) * stride + i) : 0u;
            }
#pragma unroll
        for (int j = 0; j < COMPACT_CPW; ++j)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t i = 64 * k + lane;
                if (i < n[j]) tok[(uint64_t)o[j] + i] = v[j][k];
            }
        for (int j = 0; j < COMPACT_CPW; ++j) {  // chunks with more than 256 ids
            const uint32_t *src = tokc + (cb + j) * stride;
            for (uint32_t i0 = 256; i0 < n[j]; i0 += 256) {
                uint32_t w[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t i = i0 + 64 * k + lane;
                    w[k] = i < n[j] ? __builtin_nontemporal_load(src + i) : 0u;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t i = i0 + 64 * k + lane;
                    if (i < n[j]) tok[(uint64_t)o[j] + i] = w[k];
                }
            }
        }
        return;
    }
    // byte-level BPE / unigram with long items: an entry LONG_MARK | i stands
    // for the k ids of long piece i (in long_scratch at its byte position) or
    // of pool item i; a unigram Viterbi job's entry LONG_MARK | UNI_JOB_BIT |
    // k << 24 | pos for the k u16 ids at pos of its chunk's results region.
    // The wave's chunks go in lockstep, 64 entries of each a step, so their
    // dependent loads (entry -> item -> ids) are in flight together.
    uint32_t ne[COMPACT_CPW], written[COMPACT_CPW], nemax = 0;
#pragma unroll
    for (int j = 0; j < COMPACT_CPW; ++j) {
        ne[j] = cb + j < n_chunks ? chunk_ent[cb + j] : 0u;  // entries written by the chunk kernel
        written[j] = 0;
        nemax = ne[j] > nemax ? ne[j] : nemax;
    }
    for (uint32_t e0 = 0; e0 < nemax; e0 += 64) {
        const uint32_t e = e0 + lane;
        uint32_t x[COMPACT_CPW], w[COMPACT_CPW];
#pragma unroll
        for (int j = 0; j < COMPACT_CPW; ++j)
            x[j] = e < ne[j] ? __builtin_nontemporal_load(tokc + (cb + j) * stride + e) : 0u;
#pragma unroll
        for (int j = 0; j < COMPACT_CPW; ++j) {
            const bool mark = (x[j] & 0x80000000u) != 0u;
            const bool job = long_pool && (x[j] & UNI_JOB_BIT);
            w[j] = e >= ne[j] ? 0u : !mark ? 1u : job ? (x[j] >> 24) & 63u : long_pool ? long_pool[x[j] & 0x7FFFFFFFu]
                                                                                    : long_list[x[j] & 0x7FFFFFFFu].k;
        }
#pragma unroll
        for (int j = 0; j < COMPACT_CPW; ++j) {
            const uint32_t incl = wave_incl_sum(w[j]);
            const uint32_t at = written[j] + incl - w[j];
            uint32_t *dst = tok + o[j];
            if (e < ne[j] && at < n[j]) {
                if (!(x[j] & 0x80000000u)) {
                    dst[at] = x[j];
                } else if (long_pool && (x[j] & UNI_JOB_BIT)) {  // unigram Viterbi job
                    const uint16_t *jr = reinterpret_cast<const uint16_t *>(tokc + (cb + j) * stride + UNI_JR_OFF) +
                                         (x[j] & 0xFFFu);
                    for (uint32_t q0 = 0; q0 < w[j]; q0 += 8) {  // (8 loads in flight, then 8 stores)
                        uint32_t id[8];
#pragma unroll
                        for (uint32_t r = 0; r < 8; ++r) id[r] = q0 + r < w[j] ? jr[q0 + r] : 0u;
#pragma unroll
                        for (uint32_t r = 0; r < 8; ++r)
                            if (q0 + r < w[j]) dst[at + q0 + r] = id[r];
                    }
                } else if (long_pool) {  // unigram long item: [k, ids...] in the pool
                    const uint32_t po = x[j] & 0x7FFFFFFFu;
                    for (uint32_t q = 0; q < w[j]; ++q) dst[at + q] = long_pool[po + 1 + q];
                } else {
                    const uint64_t pos = long_list[x[j] & 0x7FFFFFFFu].pos;
                    for (uint32_t q = 0; q < w[j]; ++q) dst[at + q] = long_scratch[pos + q];
                }
            }
            written[j] += (uint32_t)lane_bcast((int)incl, 63);
        }
    }
}

// ---------------------------------------------------------------------------
// Per record: where its ids start, how many, and how many rows it yields.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void record_one(const RowParams &P, const uint64_t *__restrict__ off, int64_t r, int64_t N,
                                           const uint32_t *__restrict__ chunk_off, int64_t n_chunks,
                                           const uint32_t *__restrict__ rec_local, uint32_t *__restrict__ rec_tok,
                                           uint32_t *__restrict__ rec_cnt, uint32_t *__restrict__ rec_rows) {
    auto tok_off = [&](int64_t q) -> uint32_t {
        const int64_t p = (int64_t)off[q];
        // (chunk_off[n_chunks], the total, is final once the last segment is scanned:
        // only the last segment holds records that end at N)
        return p >= N ? chunk_off[n_chunks] : chunk_off[p / CHUNK] + rec_local[q];
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

// framing id k (< MAX_FRAME) without dynamic indexing of the kernel argument
__device__ __forceinline__ int32_t frame_id(const int32_t (&a)[MAX_FRAME], int k) {
    return k == 0 ? a[0] : k == 1 ? a[1] : k == 2 ? a[2] : a[3];
}

// Row layout of k_rows: lane L owns positions 256*m + 4*L + w (w = 0..3), so
// one Philox block (4 words) is exactly one lane's keys for round m and every
// plane store is one 16-byte write per lane.
//
// Marks the k smallest (key, position) pairs of a row held as key[m][w]: a
// radix select of the k-th smallest key with wave ballots, then a
// position-ordered tie-break among keys equal to it.  The descent stops as soon
// as exactly k keys lie below the candidate (after ~log2(S) + 2 of the 32
// steps for distinct keys), which selects the same set.
template <int MR>
__device__ __forceinline__ void select_k_smallest(const uint32_t (&key)[MR][4], int k, bool (&sel)[MR][4]) {
    if (k <= 0) {
#pragma unroll
        for (int m = 0; m < MR; ++m)
#pragma unroll
            for (int w = 0; w < 4; ++w) sel[m][w] = false;
        return;
    }
    uint32_t prefix = 0;
    for (int bit = 31; bit >= 0; --bit) {
        const uint32_t cand = prefix | (1u << bit);
        int c = 0;
#pragma unroll
        for (int m = 0; m < MR; ++m)
#pragma unroll
            for (int w = 0; w < 4; ++w) c += __popcll(__ballot(key[m][w] < cand));
        if (c == k) {  // exactly the k smallest keys lie below cand: no tie to break
#pragma unroll
            for (int m = 0; m < MR; ++m)
#pragma unroll
                for (int w = 0; w < 4; ++w) sel[m][w] = key[m][w] < cand;
            return;
        }
        if (c < k) prefix = cand;
    }
    int c_lt = 0;
#pragma unroll
    for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int w = 0; w < 4; ++w) c_lt += __popcll(__ballot(key[m][w] < prefix));
    const int need = k - c_lt;
    const uint64_t lt_mask = (1ull << lane_id()) - 1ull;
    int before = 0;  // equal keys in earlier rounds
#pragma unroll
    for (int m = 0; m < MR; ++m) {
        uint64_t eq[4];
        int lower = 0;  // equal keys of this round in lower lanes
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            eq[w] = __ballot(key[m][w] == prefix);
            lower += __popcll(eq[w] & lt_mask);
        }
        int own = 0;  // equal keys of this lane at lower w
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const bool e = key[m][w] == prefix;
            sel[m][w] = key[m][w] < prefix || (e && before + lower + own < need);
            own += e ? 1 : 0;
        }
#pragma unroll
        for (int w = 0; w < 4; ++w) before += __popcll(eq[w]);
    }
}

// The same selection, usually in far fewer steps: the Philox keys are uniform,
// so an interpolation search over the key range (the next threshold guessed
// from the counts at the bracket's ends) lands on a threshold with exactly k
// keys below it in ~3-4 counts instead of the radix descent's ~log2(S) + 2.
// Any threshold with exactly k keys below it marks the same k-smallest set; a
// tie at the k-th key (no such threshold) or a slow bracket falls back to the
// radix select.
constexpr int ROWS_INTERP_STEPS = 8;
template <int MR>
__device__ __forceinline__ void select_k_smallest_interp(const uint32_t (&key)[MR][4], int k, int nvalid,
                                                         bool (&sel)[MR][4]) {
    if (k > 0 && k < nvalid) {
        uint32_t lo = 0, hi = 0xFFFFFFFFu;  // count(key < lo) = c_lo < k < c_hi ~ count(key < hi)
        int c_lo = 0, c_hi = nvalid;
#pragma unroll 1
        for (int it = 0; it < ROWS_INTERP_STEPS && hi - lo > 1u; ++it) {
            const float f = ((float)(k - c_lo) + 0.5f) / (float)(c_hi - c_lo);
            uint32_t cand = lo + (uint32_t)((float)(hi - lo) * f);
            cand = cand <= lo ? lo + 1u : cand >= hi ? hi - 1u : cand;
            cand = __builtin_amdgcn_readfirstlane(cand);
            int c = 0;
#pragma unroll
            for (int m = 0; m < MR; ++m)
#pragma unroll
                for (int w = 0; w < 4; ++w) c += __popcll(__ballot(key[m][w] < cand));
            if (c == k) {
#pragma unroll
                for (int m = 0; m < MR; ++m)
#pragma unroll
                    for (int w = 0; w < 4; ++w) sel[m][w] = key[m][w] < cand;
                return;
            }
            if (c < k) {
                lo = cand;
                c_lo = c;
            } else {
                hi = cand;
                c_hi = c;
            }
        }
    }
    select_k_smallest<MR>(key, k, sel);
}

__device__ __forceinline__ void store4(int32_t *p, int j0, int S, bool vec, int32_t a, int32_t b, int32_t c,
                                       int32_t d) {
    if (vec) {  // the planes stream out: non-temporal, they are not re-read by this pass
        typedef int32_t v4i __attribute__((ext_vector_type(4)));
        if (j0 < S) __builtin_nontemporal_store(v4i{a, b, c, d}, reinterpret_cast<v4i *>(p + j0));
    } else {
        if (j0 < S) p[j0] = a;
        if (j0 + 1 < S) p[j0 + 1] = b;
        if (j0 + 2 < S) p[j0 + 2] = c;
        if (j0 + 3 < S) p[j0 + 3] = d;
    }
}

// One row g of the call (a wave): BertData::put_data (+ mask_batch) / GptData::put_data framing and
// planes; g >= G: a padding row of the last batch.  late_bits: the row's mask words (LATE).
template <int MR, bool RM1, bool LATE>
__device__ __forceinline__ void row_one(const RowParams &P, const uint32_t *__restrict__ tok,
                                        const uint32_t *__restrict__ rec_tok, const uint32_t *__restrict__ rec_cnt,
                                        const uint32_t *__restrict__ row_off, const uint32_t *__restrict__ row_rec,
                                        int64_t g, int64_t G, const RowOut &out, const uint32_t *late_bits,
                                        int lane) {
    const int S = P.S;
    const bool vec = (S & 3) == 0;  // 16-byte aligned rows
    const bool vec_lb = (P.label_width & 3) == 0;
    const DirectDst &dd = out.direct;
    int32_t *ids_o = out.input_ids + g * S;
    int32_t *am_o = out.attention_mask + g * S;
    int32_t *tt_o = out.token_type_ids ? out.token_type_ids + g * S : nullptr;
    int32_t *lb_o = out.labels ? out.labels + g * (int64_t)P.label_width : nullptr;
    if (g < (int64_t)dd.cap) {  // a small push's row: straight into its host batch
        const uint32_t slot = dd.base + (uint32_t)g, bi = slot >= dd.B ? 1u : 0u, row = slot - bi * dd.B;
        ids_o = dd.ids[bi] + (size_t)row * S;
        am_o = dd.am[bi] + (size_t)row * S;
        tt_o = dd.tt[bi] ? dd.tt[bi] + (size_t)row * S : nullptr;
        lb_o = dd.lab[bi] ? dd.lab[bi] + (size_t)row * P.label_width : nullptr;
    }
    if (g >= (int64_t)G) {  // rows of the last batch nobody filled: initial values
#pragma unroll
        for (int m = 0; m < MR; ++m) {
            const int j0 = 256 * m + 4 * lane;
            store4(ids_o, j0, S, vec, 0, 0, 0, 0);
            store4(am_o, j0, S, vec, 1, 1, 1, 1);
            if (tt_o) store4(tt_o, j0, S, vec, 0, 0, 0, 0);
            if (lb_o) store4(lb_o, j0, P.label_width, vec_lb, -100, -100, -100, -100);
        }
        return;
    }
    const int64_t r = row_rec[g];
    const uint32_t k = (uint32_t)(g - row_off[r]);
    const uint32_t cnt = rec_cnt[r];
    const uint32_t t0 = rec_tok[r];
    const int64_t n = (int64_t)cnt + P.n_pre + P.n_post;
    const int64_t base = P.chunk ? (int64_t)k * S : 0;
    const int l = (int)((n - base) < S ? (n - base) : S);
    // (rng_mode 1) the row's mask words, one dword a lane: walked beside the tokenizer
    // (k_mask_bits_rec), else by the LATE pass (late_bits, LDS).  A row the first pass leaves to
    // the LATE one returns only after its loads are issued: the mask words' load, a dependent
    // step after row_rec / row_off, then overlaps the ids' (wave-uniform: a wave per row).
    uint32_t mwd[MR];
    bool mine = true;
    if (RM1) {
        const int64_t pre = rand_pre_slot(P, r, k);
        mine = LATE || pre >= 0;
        const uint32_t *bw = LATE ? late_bits : P.mask_bits0 + (pre >= 0 ? pre : 0) * (int64_t)P.mask_w;
#pragma unroll
        for (int m = 0; m < MR; ++m) {
            const int j0 = 256 * m + 4 * lane;
            mwd[m] = j0 < S && mine ? bw[j0 >> 5] : 0u;
        }
        if (LATE) __builtin_amdgcn_wave_barrier();  // (the LDS bits are rewritten by the wave's next rows)
    }

    int32_t id[MR][4];
#pragma unroll
    for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int j = 256 * m + 4 * lane + w;
            int32_t v = 0;
            if (j < l) {
                const int64_t f = base + j;
                if (f < P.n_pre) v = frame_id(P.pre, (int)f);
                else if (f < P.n_pre + (int64_t)cnt) v = (int32_t)tok[t0 + (f - P.n_pre)];
                else v = frame_id(P.post, (int)(f - P.n_pre - cnt));
            }
            id[m][w] = v;
        }
    if (RM1 && !mine) return;  // (the LATE pass's row)
    // attention: 0 on [S-l, S) when l < S (reversed-range quirk, bert_data.rs:58-63 / gpt_data.rs:33-41)
    const int tail0 = l < S ? S - l : S;
    const uint64_t rec = P.first_record + (uint64_t)r;
    if (P.task == 0) {  // MLM: BertData::mask_batch
        bool sel[MR][4];
        if (RM1) {  // rand-compatible mode: the row's bits from k_mask_rand
#pragma unroll
            for (int m = 0; m < MR; ++m) {
                const int j0 = 256 * m + 4 * lane;
#pragma unroll
                for (int w = 0; w < 4; ++w) sel[m][w] = (mwd[m] >> ((j0 + w) & 31)) & 1u;
            }
        } else {
            uint32_t key[MR][4];
#pragma unroll
            for (int m = 0; m < MR; ++m) {
                const uint4 c = philox4x32_10(make_uint4((uint32_t)(64 * m + lane), k, (uint32_t)rec,
                                                         (uint32_t)(rec >> 32)),
                                              (uint32_t)P.seed, (uint32_t)(P.seed >> 32));
                const int j0 = 256 * m + 4 * lane;
                key[m][0] = j0 < S ? c.x : 0xFFFFFFFFu;
                key[m][1] = j0 + 1 < S ? c.y : 0xFFFFFFFFu;
                key[m][2] = j0 + 2 < S ? c.z : 0xFFFFFFFFu;
                key[m][3] = j0 + 3 < S ? c.w : 0xFFFFFFFFu;
            }
            select_k_smallest_interp<MR>(key, P.mask_length, S < 256 * MR ? S : 256 * MR, sel);
        }
#pragma unroll
        for (int m = 0; m < MR; ++m) {
            const int j0 = 256 * m + 4 * lane;
            int32_t v[4], lab[4], am[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                v[w] = id[m][w];
                lab[w] = -100;
                if (sel[m][w] && v[w] != 0) {
                    lab[w] = v[w];
                    v[w] = P.mask_id;
                }
                am[w] = j0 + w >= tail0 ? 0 : 1;
            }
            store4(ids_o, j0, S, vec, v[0], v[1], v[2], v[3]);
            store4(am_o, j0, S, vec, am[0], am[1], am[2], am[3]);
            if (tt_o) store4(tt_o, j0, S, vec, 0, 0, 0, 0);
            store4(lb_o, j0, P.label_width, vec_lb, lab[0], lab[1], lab[2], lab[3]);
        }
    } else if (P.task == 3 || P.task == 4) {  // Multi/SingleClass: BertData::put_data rows; labels by k_*_labels
#pragma unroll
        for (int m = 0; m < MR; ++m) {
            const int j0 = 256 * m + 4 * lane;
            int32_t am[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) am[w] = j0 + w >= tail0 ? 0 : 1;
            store4(ids_o, j0, S, vec, id[m][0], id[m][1], id[m][2], id[m][3]);
            store4(am_o, j0, S, vec, am[0], am[1], am[2], am[3]);
            if (tt_o) store4(tt_o, j0, S, vec, 0, 0, 0, 0);
        }
    } else {  // CLM: GptData::put_data, labels = row as i32 (no shift)
#pragma unroll
        for (int m = 0; m < MR; ++m) {
            const int j0 = 256 * m + 4 * lane;
            int32_t am[4], lab[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const bool tail = j0 + w >= tail0;
                am[w] = tail ? 0 : 1;
                lab[w] = tail ? -100 : id[m][w];
            }
            store4(ids_o, j0, S, vec, id[m][0], id[m][1], id[m][2], id[m][3]);
            store4(am_o, j0, S, vec, am[0], am[1], am[2], am[3]);
            if (tt_o) store4(tt_o, j0, S, vec, 0, 0, 0, 0);
            store4(lb_o, j0, P.label_width, vec_lb, lab[0], lab[1], lab[2], lab[3]);
        }
    }
}

// A per-record push (<= 64 records, <= 64 chunks): the same steps on one wave -- wave scans, no
// workgroup barriers.  With the rows fused (MR > 0: nothing after this kernel reads the call's
// record / row tables) those tables live in LDS, so the only global round trip between steps is
// the compacted ids (a push is bound by such dependent round trips: 10.6 us with every table in
// global memory).  Lane order is program order within the wave; a fence between steps makes one
// lane's writes visible to the others' reads.
template <int MR>
__device__ __forceinline__ void downstream_tiny(const SmallDown &d, const RowParams &P, const uint64_t *__restrict__ off,
                                                int64_t R, int64_t N, int64_t n_chunks) {
    constexpr int ROWS_LDS = 1024;
    __shared__ uint32_t s_coff[65], s_rtok[64], s_rcnt[64], s_rrows[64], s_roff[65];
    __shared__ uint32_t s_rrec[MR > 0 ? ROWS_LDS : 1];
    const int lane = lane_id();
    auto step = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
    uint32_t *const coff = MR > 0 ? s_coff : d.chunk_off;
    uint32_t *const rtok = MR > 0 ? s_rtok : d.rec_tok, *const rcnt = MR > 0 ? s_rcnt : d.rec_cnt;
    uint32_t *const rrows = MR > 0 ? s_rrows : d.rec_rows, *const roff = MR > 0 ? s_roff : d.row_off;
    {
        const uint32_t c = lane < n_chunks ? d.chunk_cnt[lane] : 0u;
        const uint32_t incl = wave_incl_sum(c);
        if (lane < n_chunks) coff[lane] = incl - c;
        if (lane == 63) coff[n_chunks] = incl;
    }
    step();
    // (the records' loads before the compaction's stores: independent, in flight together)
    if (lane < R) record_one(P, off, lane, N, coff, n_chunks, d.rec_local, rtok, rcnt, rrows);
    for (int64_t cb = 0; cb < n_chunks; cb += COMPACT_CPW)
        compact_wave(cb, d.tokc, d.chunk_cnt, coff, n_chunks, d.tok, d.long_count, d.chunk_ent, d.long_list,
                     d.long_scratch, d.long_pool, d.stride);
    step();
    uint32_t G;
    {
        const uint32_t c = lane < R ? rrows[lane] : 0u;
        const uint32_t incl = wave_incl_sum(c);
        G = (uint32_t)lane_bcast((int)incl, 63);
        if (lane < R) roff[lane] = incl - c;
        if (lane == 63) roff[R] = incl;
        uint32_t *const rrec = MR > 0 && G <= (uint32_t)ROWS_LDS ? s_rrec : d.row_rec;
        if (lane < R)
            for (uint32_t g = incl - c; g < incl; ++g) rrec[g] = (uint32_t)lane;
        if (d.stat) {
            if (lane < R) d.stat[lane] = incl - c;
            if (lane == 63) {
                d.stat[R] = incl;
                d.stat[R + 1] = 0u;
                d.stat[R + 2] = d.tok_err ? *d.tok_err : 0u;  // a t5 tokenizer under mlm / clm
            }
        }
    }
    if constexpr (MR > 0) {
        step();
        const uint32_t *const rrec = G <= (uint32_t)ROWS_LDS ? s_rrec : d.row_rec;
        const int64_t g_end = d.out.direct.cap ? (int64_t)G : ((int64_t)G + P.B - 1) / P.B * P.B;
        for (int64_t g = 0; g < g_end; ++g)
            row_one<MR, false, false>(P, d.tok, rtok, rcnt, roff, rrec, g, (int64_t)G, d.out, nullptr, lane);
    }
}

}  // namespace sdl
