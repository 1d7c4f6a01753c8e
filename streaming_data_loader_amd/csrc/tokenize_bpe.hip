// tokenize_bpe.hip -- GPT-2 byte-level BPE tokenization of a text arena on gfx950.
//
// Restates, for a whole arena of records at once, what the reference does one
// record at a time for task=clm (TokenizerHolder::get_ids ->
// tokenizers::Tokenizer::encode, rust/src/tokenizer/tokenizer_holder.rs:19-28;
// crate tokenizers 0.13.1) with the gpt2 tokenizer.json:
//   AddedVocabulary split (<|endoftext|> on the raw text)
//   -> ByteLevel pre-tokenizer, GPT-2 regex
//        's|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+
//   -> BPE by merge rank on the byte-level symbols of every pre-token.
// The wrapper's [eos] ... [eos] framing is added at row assembly (pipeline.hip).
//
// The regex is evaluated byte-parallel: whether a pre-token starts at a char
// depends only on a few neighbouring chars (previous char class, contraction
// letters, whether a whitespace char ends its run), so every lane flags the
// starts among its 16 bytes from the chunk's LDS window and class array.
//
// One wave64 per workgroup owns CHUNK bytes (16 per lane), as the WordPiece
// kernel, and produces the same outputs (per-chunk id list in `tokc`, count,
// per-record local offsets), so scans, compaction and rows are shared:
//   1. load the window; classify every byte (ASCII arithmetically; lead bytes
//      block-parallel through the probed class table; added tokens);
//   2. pre-token starts -> LDS piece list;
//   3. each piece: one probe of the word table (every vocab string whose BPE
//      is itself, keyed by raw bytes) -- nearly every pre-token ends here;
//   4. misses of <= 64 bytes: wave-cooperative BPE, one lane per symbol: each
//      step merges every occurrence of the lowest-ranked adjacent pair (left
//      to right within overlapping runs), the order tokenizers' heap yields
//      for rank-monotone merges (checked on the host);
//   5. longer pieces (or pieces running past the window) are appended to a
//      global list and finished by k_bpe_long; the chunk list holds a marker.
#include <algorithm>

#include "common.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "tok_device.hpp"

namespace sdl {

namespace {

// per-byte class in LDS
// (one bit per class, continuation bytes 0: the start rules run byte-parallel)
enum : uint8_t { K_CONT = 0, K_L = 1, K_N = 2, K_W = 4, K_SP = 8, K_AP = 0x10, K_O = 0x20, K_SPEC = 0x40, K_SPX = 0x80 };
constexpr int K_BND = 15;  // "no char" (record start / added-token edge / text end)
constexpr int BPE_MAX_WAVE = 64;  // pieces up to this many bytes are merged in the chunk kernel
constexpr uint8_t CNT_LONG = 0xFF;  // s_cnt of a long piece (k_bpe_long)
constexpr uint32_t LONG_MARK = 0x80000000u;

__device__ __forceinline__ uint32_t ascii_k(uint32_t b) {
    if ((b | 0x20u) - 'a' < 26u) return K_L;
    if (b - '0' < 10u) return K_N;
    if (b == ' ') return K_SP;
    if (b - 9u < 5u) return K_W;
    if (b == '\'') return K_AP;
    return K_O;
}

// ascii_k of 4 bytes (bytes >= 0x80: K_O)
__device__ __forceinline__ uint32_t ascii_k4(uint32_t x) {
    const uint32_t lo7 = ~(x & B7), a = x & 0x7F7F7F7Fu;
    const uint32_t l = in7(a | 0x20202020u, 'a', 'z') & lo7, n = in7(a, '0', '9') & lo7, w = in7(a, 9, 13) & lo7,
                   sp = in7(a, ' ', ' ') & lo7, ap = in7(a, '\'', '\'') & lo7;
    const uint32_t o = B7 & ~(l | n | w | sp | ap);
    return (l >> 7) | (n >> 6) | (w >> 5) | (sp >> 4) | (ap >> 3) | (o >> 2);
}

__device__ __forceinline__ uint32_t gclass(const DevTok &T, uint32_t cp) {
    if (cp >= 0x110000u) return GC_O;
    return (T.gblock[(uint32_t)T.gpage[cp >> 8] * 64u + ((cp & 255u) >> 2)] >> (2 * (cp & 3u))) & 3u;
}

__device__ __forceinline__ uint32_t k_of_gc(uint32_t g) {
    return g == GC_L ? K_L : g == GC_N ? K_N : g == GC_W ? K_W : K_O;
}

__device__ __forceinline__ bool is_w(int k) { return k == K_W || k == K_SP; }

// rank/merged id of the pair (a, b): one cuckoo probe (two 8-B loads)
__device__ __forceinline__ uint32_t merge_val(const DevTok &T, uint32_t a, uint32_t b) {
    const uint32_t key = a << 16 | b, h = merge_hash(key);
    const MSlot s1 = T.mslots[cuckoo_slot1(h, T.mslot_mask)];
    const MSlot s2 = T.mslots[cuckoo_slot2(h, T.mslot_mask)];
    if (s1.key == key) return s1.val;
    if (s2.key == key) return s2.val;
    return 0xFFFFFFFFu;
}

__device__ __forceinline__ uint32_t min_u32(uint32_t a, uint32_t b) { return a < b ? a : b; }
// wave minimum: a DPP min-scan, lane 63's total read back (no ds_bpermute steps)
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
    DPP_SCAN_ID(x, min_u32, 0xFFFFFFFFu);
    return lane_bcast(x, 63);
}
// segmented min-scan operator on (head flag << 16 | rank <= 0xFFFF): a head
// starts a new segment (its own value stands), else the running min carries
// and so does "a head was seen"
__device__ __forceinline__ uint32_t seg_min(uint32_t a, uint32_t b) {
    return (b & 0x10000u) ? b : ((a & 0x10000u) | min_u32(a & 0xFFFFu, b & 0xFFFFu));
}

// Of the candidate pairs in m (bit j = pair (j, j+1)), those merged left to
// right: the first of every run of adjacent candidates, then every other one.
__device__ __forceinline__ uint64_t leftmost_alternating(uint64_t m, bool blocked0) {
    uint64_t sel = 0;
    if (blocked0) m &= ~1ull;  // its left symbol was merged into the previous pair
    while (m) {
        const uint64_t s = m & ~(m << 1);
        sel |= s;
        m &= ~(s | (s << 1));
    }
    return sel;
}

// ---- the GPT-2 regex as local rules --------------------------------------------
// A pre-token starts at the char at q iff (pc = class of the previous char,
// BND at a record start or next to an added token):
//   added token                       -> start
//   pc == BND                         -> start
//   whitespace c: pc not whitespace   -> start
//                 else start iff the next char is neither whitespace nor BND
//                 (\s+(?!\S) leaves the last whitespace of a run to the next
//                 pre-token)
//   pc == ' '                         -> no  (" ?" prefix of L/N/O runs)
//   pc other whitespace               -> start
//   ' (apostrophe): start iff pc is a letter or digit
//   O: start iff pc is not O/'
//   N: start iff pc is not N
//   L: after an apostrophe: start iff that apostrophe does not begin a
//      contraction; after L: start iff a contraction ends right before q;
//      else start.
// A contraction ('s 't 're 've 'm 'll 'd, case-sensitive) begins at an
// apostrophe that itself begins a pre-token: pc is BND, L, N or non-space
// whitespace.  Every char is a valid UTF-8 sequence or one O byte.

// Accessor over the chunk's LDS window (positions are window indices).
struct LdsAcc {
    const lds_u8 *win;
    const lds_u8 *cls;
    const lds_u32 *rbits;
    int64_t w0, N;
    __device__ __forceinline__ int k(int q) const { return cls[q]; }
    __device__ __forceinline__ uint32_t b(int q) const { return win[q]; }
    __device__ __forceinline__ bool rs(int q) const { return (rbits[q >> 5] >> (q & 31)) & 1u; }
    __device__ __forceinline__ bool past(int q) const { return q >= WIN || w0 + q >= N; }
};

// Class of the byte at absolute position q computed from global memory (the
// long-piece path).  Added tokens are ASCII (checked on the host), so no
// UTF-8 sequence overlaps one.
__device__ int gk_of(const Ctx &C, int64_t q) {
    const DevTok &T = *C.T;
    if (q < 0 || q >= C.N) return K_O;
    if (T.n_special) {
        for (int d = 0; d < T.max_special_len && q - d >= 0; ++d) {
            const int64_t x = q - d;
            if (C.byte(x) == T.opener) {
                const int m = special_match(C, x);
                if (m >= 0 && T.special_len[m] > d) return d == 0 ? K_SPEC : K_SPX;
            }
            if (C.rstart(x)) break;
        }
    }
    const uint32_t b = C.byte(q);
    if (b < 0x80u) return (int)ascii_k(b);
    int len;
    if (b >= 0xC0u) {
        const uint32_t cp = decode(C, q, b, &len);
        return len == 1 ? K_O : (int)k_of_gc(gclass(T, cp));
    }
    for (int d = 1; d <= 3 && q - d >= 0; ++d) {  // covered by a lead within 3 bytes?
        if (C.rstart(q - d + 1)) break;
        const uint32_t x = C.byte(q - d);
        if ((x & 0xC0u) == 0x80u) continue;
        if (x < 0xC0u) break;
        decode(C, q - d, x, &len);
        return len > d ? K_CONT : K_O;
    }
    return K_O;
}

struct GlobAcc {
    const Ctx *C;
    __device__ __forceinline__ int k(int64_t q) const { return gk_of(*C, q); }
    __device__ __forceinline__ uint32_t b(int64_t q) const { return C->byte(q); }
    __device__ __forceinline__ bool rs(int64_t q) const { return C->rstart(q); }
    __device__ __forceinline__ bool past(int64_t q) const { return q >= C->N; }
};

// class of the char before the one at q; *pq = its position
template <class A, class P>
__device__ __forceinline__ int prev_k(const A &a, P q, P *pq) {
    if (a.rs(q)) return K_BND;
    P x = q - 1;
    int k = a.k(x);
    for (int s = 0; s < 3 && k == K_CONT; ++s) k = a.k(--x);
    *pq = x;
    return (k == K_SPEC || k == K_SPX) ? K_BND : k;
}
// class of the char after the one at q
template <class A, class P>
__device__ __forceinline__ int next_k(const A &a, P q) {
    P x = q + 1;
    for (int s = 0; s < 3 && !a.past(x) && a.k(x) == K_CONT; ++s) ++x;
    if (a.past(x) || a.rs(x)) return K_BND;
    const int k = a.k(x);
    return k == K_SPEC ? K_BND : k;
}
// length (2 or 3) of the contraction beginning at the apostrophe q, else 0
template <class A, class P>
__device__ __forceinline__ int contraction(const A &a, P q) {
    P pq;
    const int pk = prev_k(a, q, &pq);
    if (!(pk == K_BND || pk == K_L || pk == K_N || pk == K_W)) return 0;
    if (a.past(q + 1) || a.rs(q + 1) || a.k(q + 1) != K_L) return 0;
    const uint32_t b1 = a.b(q + 1);
    if (b1 == 's' || b1 == 't' || b1 == 'm' || b1 == 'd') return 2;
    if (a.past(q + 2) || a.rs(q + 2) || a.k(q + 2) != K_L) return 0;
    const uint32_t b2 = a.b(q + 2);
    if ((b1 == 'r' && b2 == 'e') || (b1 == 'v' && b2 == 'e') || (b1 == 'l' && b2 == 'l')) return 3;
    return 0;
}
template <class A, class P>
__device__ bool is_start(const A &a, P q) {
    const int c = a.k(q);
    if (c == K_CONT || c == K_SPX) return false;
    if (c == K_SPEC) return true;
    P pq = q - 1;
    const int pc = prev_k(a, q, &pq);
    if (pc == K_BND) return true;
    if (is_w(c)) {
        if (!is_w(pc)) return true;
        const int nk = next_k(a, q);
        return !(is_w(nk) || nk == K_BND);
    }
    if (pc == K_SP) return false;
    if (pc == K_W) return true;
    switch (c) {
        case K_AP: return pc == K_L || pc == K_N;
        case K_O: return !(pc == K_O || pc == K_AP);
        case K_N: return pc != K_N;
        default: break;  // K_L
    }
    if (pc == K_AP) return contraction(a, pq) == 0;
    if (pc != K_L) return true;
    if (a.k(q - 2) == K_AP && !a.rs(q - 1) && contraction(a, q - 2) == 2) return true;
    if (a.k(q - 3) == K_AP && !a.rs(q - 2) && !a.rs(q - 1) && contraction(a, q - 3) == 3) return true;
    return false;
}

// End of the piece starting at p when it runs past its chunk's window: the
// next pre-token start, record start or the text end (wave-parallel scan).
__device__ int64_t bpe_piece_end(const Ctx &C, int64_t p) {
    const GlobAcc a{&C};
    const int lane = lane_id();
    for (int64_t q0 = p + 1;; q0 += 64) {
        const int64_t q = q0 + lane;
        const bool hit = q >= C.N || C.rstart(q) || is_start(a, q);
        const uint64_t m = __ballot(hit);
        if (m) return q0 + __builtin_ctzll(m);
    }
}

// Wave-cooperative BPE of n <= 64 byte symbols held one per lane (sym valid on
// lanes < n).  Returns the final symbol count; lane j < count holds id j.
__device__ int bpe_wave(const DevTok &T, uint32_t &sym, int n, lds_u16 *tmp) {
    const int lane = lane_id();
    const uint64_t lt = (1ull << lane) - 1ull;
    while (n > 1) {
        const uint32_t nxt = wave_next(sym);
        const uint32_t v = lane < n - 1 ? merge_val(T, sym, nxt) : 0xFFFFFFFFu;
        const uint32_t rank = v >> 16;
        const uint32_t rmin = wave_min_u32(rank);
        if (rmin == 0xFFFFu) break;
        const uint64_t cand = __ballot(rank == rmin && lane < n - 1);
        const uint64_t sel = leftmost_alternating(cand, false);
        const bool me_sel = (sel >> lane) & 1ull;
        if (me_sel) sym = v & 0xFFFFu;
        const uint64_t live = (n == 64 ? ~0ull : ((1ull << n) - 1ull)) & ~(sel << 1);
        if ((live >> lane) & 1ull) tmp[__popcll(live & lt)] = (uint16_t)sym;
        __builtin_amdgcn_wave_barrier();
        n = __popcll(live);
        sym = lane < n ? tmp[lane] : 0u;
        __builtin_amdgcn_wave_barrier();
    }
    return n;
}

// Segmented form: lanes < n hold the byte symbols of several words, each word
// a run of lanes starting at a set bit of `heads` (bit 0 set).  Every word
// runs bpe_wave's steps independently and at once: per word the lowest rank
// among its adjacent pairs, all its non-overlapping occurrences merged left to
// right.  Pairs never straddle a word, so the runs of candidate bits do not
// either and one leftmost_alternating serves every word.  Returns the final
// symbol count; `heads` then marks where each word's ids start.
//
// A pair's merge value travels with its left symbol through the compaction; only
// the pairs a step changed -- a merged symbol's, and its left neighbour's -- are
// probed again (each probe is an L2 round trip on the step's critical path).
__device__ int bpe_wave_seg(const DevTok &T, uint32_t &sym, int n, uint64_t &heads, lds_u32 *tmp, lds_u32 *tmpv) {
    const int lane = lane_id();
    const uint64_t lt = (1ull << lane) - 1ull;
    bool need = true;  // this lane's pair value is not known
    uint32_t vk = 0;   // ... or this
    for (;;) {
        const uint32_t nxt = wave_next(sym);
        const bool pair = lane < n - 1 && !((heads >> (lane + 1)) & 1ull);
        const uint32_t v = !pair ? 0xFFFFFFFFu : need ? merge_val(T, sym, nxt) : vk;
        const uint32_t rank = v >> 16;
        // segmented inclusive min scan (DPP), then each lane takes its word's last value
        uint32_t x = rank | ((uint32_t)((heads >> lane) & 1ull) << 16);
        DPP_SCAN_ID(x, seg_min, 0xFFFFu);
        x &= 0xFFFFu;
        const uint64_t after = lane == 63 ? 0ull : heads & ~((2ull << lane) - 1ull);
        const int last = after ? __builtin_ctzll(after) - 1 : n - 1;
        const uint32_t rmin = (uint32_t)__shfl((int)x, last < 0 ? 0 : last, 64);
        if (!__any(lane < n && rmin != 0xFFFFu)) break;
        const uint64_t cand = __ballot(pair && rank == rmin && rank != 0xFFFFu);
        const uint64_t sel = leftmost_alternating(cand, false);
        if ((sel >> lane) & 1ull) sym = v & 0xFFFFu;
        const uint64_t live = (n == 64 ? ~0ull : ((1ull << n) - 1ull)) & ~(sel << 1);
        // heads are never merged away (no pair straddles one): each travels with
        // its symbol through the compaction and is re-balloted at its new lane
        // the pair changes for a merged symbol and for the lane left of one
        const bool nd = ((sel >> lane) & 1ull) || (lane < 63 && ((sel >> (lane + 1)) & 1ull));
        if ((live >> lane) & 1ull) {
            const int at = __popcll(live & lt);
            tmp[at] = (sym & 0xFFFFu) | (uint32_t)((heads >> lane) & 1ull) << 16 | (nd ? 1u : 0u) << 17;
            tmpv[at] = v;
        }
        __builtin_amdgcn_wave_barrier();
        n = __popcll(live);
        const uint32_t w = lane < n ? tmp[lane] : 0u;
        sym = w & 0xFFFFu;
        heads = __ballot((w >> 16) & 1u);
        need = ((w >> 17) & 1u) != 0u;
        vk = lane < n ? tmpv[lane] : 0xFFFFFFFFu;
        __builtin_amdgcn_wave_barrier();
    }
    return n;
}

// One word of 2..LANE_BPE byte symbols per lane, tokenizers' order: BPE::merge_word pops its
// heap of (rank, position), i.e. the lowest-rank pair, leftmost among equal ranks, one merge at a
// time.  The symbols and their pairs' merge values stay in registers (static indices: a merge at
// lane-varying j is a select per slot); only the two pairs a merge creates are probed again.  A
// wave runs 64 words at once and pays the longest word's merge count in probe latencies, where
// the segmented wave BPE pays every packed batch's.  s[0 .. returned count) = the word's ids.
constexpr int LANE_BPE = 12;  // (16: held-out clm -1.3 %, fixture -1.7 %: its registers cost the common path; 8: held-out -3.5 %)
__device__ __forceinline__ int bpe_lane(const DevTok &T, uint32_t (&s)[LANE_BPE], int n) {
    constexpr uint32_t NOV = 0xFFFFFFFFu;
    uint32_t v[LANE_BPE - 1];
#pragma unroll
    for (int k = 0; k < LANE_BPE - 1; ++k) v[k] = k < n - 1 ? merge_val(T, s[k], s[k + 1]) : NOV;
    for (;;) {
        // the lowest rank, leftmost on ties (strict <, ascending k)
        uint32_t br = 0xFFFFu, bv = 0;
        int j = -1;
#pragma unroll
        for (int k = 0; k < LANE_BPE - 1; ++k) {
            const uint32_t r = v[k] >> 16;
            const bool lt = r < br;
            br = lt ? r : br;
            bv = lt ? v[k] : bv;
            j = lt ? k : j;
        }
        if (!__any(j >= 0)) break;
        if (j >= 0) {
            const uint32_t m = bv & 0xFFFFu;
            uint32_t left = 0, right = 0;  // the symbols beside the merged pair
#pragma unroll
            for (int k = 0; k < LANE_BPE; ++k) {
                left = k == j - 1 ? s[k] : left;
                right = k == j + 2 ? s[k] : right;
            }
#pragma unroll
            for (int k = 0; k < LANE_BPE; ++k) {
                const uint32_t nx = k + 1 < LANE_BPE ? s[k + 1] : 0u;
                s[k] = k < j ? s[k] : k == j ? m : nx;
            }
#pragma unroll
            for (int k = 0; k < LANE_BPE - 1; ++k) {
                const uint32_t nx = k + 1 < LANE_BPE - 1 ? v[k + 1] : NOV;
                v[k] = k < j - 1 ? v[k] : k <= j ? NOV : nx;
            }
            --n;
            // the two new pairs: (left, m) at j - 1 and (m, right) at j
            const uint32_t vl = j > 0 ? merge_val(T, left, m) : NOV;
            const uint32_t vr = j < n - 1 ? merge_val(T, m, right) : NOV;
#pragma unroll
            for (int k = 0; k < LANE_BPE - 1; ++k) v[k] = k == j - 1 ? vl : k == j ? vr : v[k];
        }
    }
    return n;
}

}  // namespace

// Diagnostic build (-DSDL_STAMPS): lane 0 of every block adds the s_memtime
// cycles between phase boundaries into sdl_bpe_cycles[]; never in the product.
#ifdef SDL_STAMPS
__device__ unsigned long long sdl_bpe_cycles[8];
#define BPE_STAMP(k)                                                                  \
    do {                                                                              \
        if (threadIdx.x == 0) {                                                       \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();              \
            atomicAdd(&sdl_bpe_cycles[k], t_ - stamp_prev_);                          \
            stamp_prev_ = t_;                                                         \
        }                                                                             \
    } while (0)
void print_bpe_cycles() {
    unsigned long long h[8];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(sdl_bpe_cycles), sizeof(h)) != hipSuccess) return;
    static const char *names[] = {"", "load+classify", "pre-token starts", "word-table probes", "wave BPE",
                                  "compact", "lane BPE", "-"};
    unsigned long long tot = 0;
    for (int i = 1; i < 7; ++i) tot += h[i];
    for (int i = 1; i < 7; ++i)
        fprintf(stderr, "[bpe stamps] %-18s %6.2f%%\n", names[i], tot ? 100.0 * (double)h[i] / (double)tot : 0.0);
}
#else
#define BPE_STAMP(k) do {} while (0)
#endif

// ---------------------------------------------------------------------------
// Register budget for 5 waves/SIMD (the 7.9 KB of LDS per one-wave block admits 5).
constexpr int BPE_WAVES = 5;
__global__ __launch_bounds__(TOK_THREADS) __attribute__((amdgpu_waves_per_eu(BPE_WAVES, 8))) void k_bpe_chunks(
    DevTok T, const uint8_t *__restrict__ text, int64_t N, const uint64_t *__restrict__ off, int64_t R,
    const uint32_t *__restrict__ ranges, uint32_t *__restrict__ tokc, uint32_t *__restrict__ chunk_cnt,
    uint32_t *__restrict__ chunk_ent, uint32_t *__restrict__ rec_local, uint32_t *__restrict__ long_count,
    BpeLong *__restrict__ long_list, uint32_t long_cap) {
    __shared__ __attribute__((aligned(16))) uint8_t s_wc[2 * WIN];  // text window | byte classes
    uint8_t *const s_win = s_wc;
    uint8_t *const s_cls = s_wc + WIN;
    __shared__ uint32_t s_rbits[RBITS_WORDS + 1];
    __shared__ uint16_t s_pieces[CHUNK + 1];  // prel | SPEC << 12 | LONG << 13
    __shared__ uint16_t s_stage[STAGE];       // ids staged at their piece's byte position
    __shared__ uint8_t s_cnt[CHUNK];          // ids per piece (<= BPE_MAX_WAVE), CNT_LONG = long piece
    __shared__ uint32_t s_tmp[64];
    __shared__ uint32_t s_tmpv[64];  // bpe_wave_seg: pair values travelling with their symbols
    __shared__ uint32_t s_scratch[8];

    const int tid = threadIdx.x;
#ifdef SDL_STAMPS
    unsigned long long stamp_prev_ = __builtin_amdgcn_s_memtime();
#endif
    const int lane = tid;
    const int64_t ci = xcd_chunk();  // this block's chunk
    const int64_t c0 = ci * CHUNK;
    const int64_t c1 = c0 + CHUNK < N ? c0 + CHUNK : N;
    const int64_t w0 = c0 - HALO_L;
    const lds_u8 *win = (const lds_u8 *)s_win;
    lds_u8 *cls = (lds_u8 *)s_cls;
    const lds_u32 *rbits = (const lds_u32 *)s_rbits;

    // ---- 1. load + classify --------------------------------------------------
    const uint4 v = load16(text, c0 + 16 * tid, N);
    *reinterpret_cast<uint4 *>(s_win + HALO_L + 16 * tid) = v;
    uint4 hv = make_uint4(0, 0, 0, 0);
    int64_t hp = 0;
    if (tid < (WIN - CHUNK) / 16) {
        hp = tid < HALO_L / 16 ? w0 + 16 * tid : c0 + CHUNK + 16 * (tid - HALO_L / 16);
        hv = load16(text, hp, N);
        *reinterpret_cast<uint4 *>(s_win + (hp - w0)) = hv;
    }
    if (tid <= RBITS_WORDS) s_rbits[tid] = 0;
    const int64_t ra = ranges[3 * ci], rz = ranges[3 * ci + 1], r_lo = ranges[3 * ci + 2];
    const int nrb = (int)(rz - ra);
    if (tid == 0) s_scratch[0] = s_scratch[1] = 0;
    __syncthreads();
    for (int k = tid; k < nrb; k += TOK_THREADS) {
        const int rel = (int)((int64_t)off[ra + k] - w0);
        atomicOr(&s_rbits[rel >> 5], 1u << (rel & 31));
    }
    // ASCII classes (bytes >= 0x80 provisionally O; text past N is O too)
    auto classify16 = [&](const uint4 &x, int wi0, int64_t p0) {
        (void)p0;
        *reinterpret_cast<uint4 *>(s_cls + wi0) = make_uint4(ascii_k4(x.x), ascii_k4(x.y), ascii_k4(x.z), ascii_k4(x.w));
    };
    classify16(v, HALO_L + 16 * tid, c0 + 16 * tid);
    if (tid < (WIN - CHUNK) / 16) classify16(hv, (int)(hp - w0), hp);
    __syncthreads();

    const Ctx C{&T, win, rbits, w0, text, N, off, R};
    // rare bytes: each lane finds its own 16 bytes' (and halo bytes') lead bytes
    // and added-token openers in registers and handles only those -- lead bytes
    // (decode: class, and the continuation bytes they cover), then added tokens
    // (override)
    auto rare_masks = [&](const uint4 &x, uint32_t &leads, uint32_t &opens) {
        leads = gather16(x.x & (x.x << 1), x.y & (x.y << 1), x.z & (x.z << 1), x.w & (x.w << 1));  // >= 0xC0
        const uint32_t o4 = T.opener * 0x01010101u;
        opens = gather16(~nzb(x.x ^ o4), ~nzb(x.y ^ o4), ~nzb(x.z ^ o4), ~nzb(x.w ^ o4));
    };
    uint32_t lead_m, open_m, hlead_m = 0, hopen_m = 0;
    rare_masks(v, lead_m, open_m);
    if (tid < (WIN - CHUNK) / 16) rare_masks(hv, hlead_m, hopen_m);
    auto do_leads = [&](uint32_t m, int wi0) {
        for (; m; m &= m - 1) {
            const int wi = wi0 + __builtin_ctz(m);
            const int64_t p = w0 + wi;
            if (p < 0 || p >= N) continue;
            int len;
            const uint32_t cp = decode(C, p, win[wi], &len);
            if (len == 1) continue;  // malformed: a one-byte O char
            cls[wi] = (uint8_t)k_of_gc(gclass(T, cp));
            for (int k = 1; k < len && wi + k < WIN; ++k) cls[wi + k] = K_CONT;
        }
    };
    do_leads(lead_m, HALO_L + 16 * tid);
    if (hlead_m) do_leads(hlead_m, (int)(hp - w0));
    __syncthreads();
    if (T.n_special) {
        auto do_opens = [&](uint32_t m, int wi0) {
            for (; m; m &= m - 1) {
                const int wi = wi0 + __builtin_ctz(m);
                const int64_t p = w0 + wi;
                if (p < 0 || p >= N) continue;
                const int mt = special_match(C, p);
                if (mt < 0) continue;
                const int l = T.special_len[mt];
                cls[wi] = K_SPEC;
                for (int j = 1; j < l && wi + j < WIN; ++j) cls[wi + j] = K_SPX;
            }
        };
        do_opens(open_m, HALO_L + 16 * tid);
        if (hopen_m) do_opens(hopen_m, (int)(hp - w0));
        __syncthreads();
    }

    BPE_STAMP(1);
    // ---- 2. pre-token starts -------------------------------------------------
    const LdsAcc A{win, cls, rbits, w0, N};
    const int64_t s0 = c0 + 16 * tid;
    const int nown = s0 >= c1 ? 0 : (int)(c1 - s0 < 16 ? c1 - s0 : 16);
    // the rules over the lane's class bytes in registers; bytes whose rule looks
    // further (apostrophes, a multi-byte previous char, whitespace before a
    // continuation byte) take is_start
    const int wi0 = HALO_L + 16 * tid;
    const uint4 kc = *reinterpret_cast<const uint4 *>(s_cls + wi0);
    const uint32_t kw[6] = {*reinterpret_cast<const uint32_t *>(s_cls + wi0 - 4), kc.x, kc.y, kc.z, kc.w,
                            *reinterpret_cast<const uint32_t *>(s_cls + wi0 + 16)};
    const uint64_t rb = ((uint64_t)s_rbits[(wi0 >> 5) + 1] << 32 | s_rbits[wi0 >> 5]) >> (wi0 & 31);
    // byte-parallel over 4 bytes per dword, each predicate in bit 7 of its byte
    constexpr uint32_t H = B7;
    const int64_t lim64 = N - s0 - 1;  // bytes i >= lim: the next byte is past the text
    const int lim = lim64 < 0 ? 0 : lim64 > 16 ? 16 : (int)lim64;
    const uint32_t rsq_bits = (uint32_t)rb & 0xFFFFu;
    const uint32_t bndn_bits = ((uint32_t)(rb >> 1) | (0xFFFFu << lim)) & 0xFFFFu;
    uint32_t fmask = 0, cmask = 0;
#pragma unroll
    for (int j = 1; j <= 4; ++j) {
        const uint32_t c = kw[j], lo = kw[j - 1];
        const uint32_t p = __builtin_amdgcn_alignbyte(c, lo, 3), p2 = __builtin_amdgcn_alignbyte(c, lo, 2),
                       p3 = __builtin_amdgcn_alignbyte(c, lo, 1);
        const uint32_t n = __builtin_amdgcn_alignbyte(kw[j + 1], c, 1);
        // class of the previous char (a continuation byte's lead is <= 3 bytes back)
        const uint32_t pe = p | (~fullb(nzb(p)) & (p2 | (~fullb(nzb(p2)) & (p3 | (~fullb(nzb(p3)) & lo)))));
        const uint32_t rsq = expand4((rsq_bits >> (4 * (j - 1))) & 0xFu);
        const uint32_t bndn = expand4((bndn_bits >> (4 * (j - 1))) & 0xFu) | bit7(n, 6);
        const uint32_t dead = (~nzb(c) & H) | bit7(c, 7);  // CONT, SPX: never a start
        const uint32_t spec = bit7(c, 6);
        const uint32_t bnd = rsq | nzb(pe & 0xC0C0C0C0u);  // pc is BND
        const uint32_t wc = nzb(c & 0x0C0C0C0Cu), wp = nzb(pe & 0x0C0C0C0Cu), wn = nzb(n & 0x0C0C0C0Cu);
        const uint32_t contn = ~nzb(n) & H;
        const uint32_t lc = bit7(c, 0), app = bit7(pe, 4);
        // left to is_start: L after an apostrophe or after L after one, whitespace
        // run before a multi-byte char
        const uint32_t cx = (lc & app) | (lc & bit7(pe, 0) & bit7(p2 | p3, 4)) | (wc & wp & contn);
        const uint32_t st = (wc & (~wp | (~bndn & ~wn & ~contn))) | (bit7(c, 4) & nzb(pe & 0x07070707u)) |
                            (nzb(c & ~pe & 0x23232323u) & ~bit7(pe, 3) & ~(app & bit7(c, 5)));
        const uint32_t live = ~dead & ~spec & ~bnd & H;
        fmask |= gather4(spec | (~dead & bnd & H) | (st & live & ~cx)) << (4 * (j - 1));
        cmask |= gather4(cx & live) << (4 * (j - 1));
    }
    const uint32_t own = nown >= 16 ? 0xFFFFu : (1u << nown) - 1u;
    uint32_t pmask = fmask & own;
    for (uint32_t m = cmask & own; m; m &= m - 1) {
        const int i = __builtin_ctz(m);
        if (is_start(A, wi0 + i)) pmask |= 1u << i;
    }
    uint32_t np_total;
    uint32_t pbase = block_excl_sum<TOK_THREADS>((uint32_t)__builtin_popcount(pmask), &np_total, s_scratch + 2);
    for (uint32_t m = pmask; m;) {
        const int i = __builtin_ctz(m);
        m &= m - 1;
        const int wi = HALO_L + 16 * tid + i;
        s_pieces[pbase++] = (uint16_t)((16 * tid + i) | (cls[wi] == K_SPEC ? 1u << 12 : 0u));
    }
    // end of the last piece: the first start at or after c1 within the window
    // (lookahead of a char needs 4 more bytes), else it runs on (long piece)
    if (tid == 0) {
        int e = -1;
        if (c1 >= N) e = (int)(c1 - c0);
        else {
            for (int wi = (int)(c1 - w0); wi < WIN - 8; ++wi) {
                if (w0 + wi >= N) { e = (int)(N - c0); break; }
                if (rbits[wi >> 5] >> (wi & 31) & 1u || is_start(A, wi)) { e = wi - HALO_L; break; }
            }
        }
        s_scratch[0] = (uint32_t)e;
    }
    __syncthreads();
    const int np = (int)np_total;
    const int e_last = (int)s_scratch[0];
    s_pieces[np] = (uint16_t)(e_last < 0 ? 0xFFFFu : (uint32_t)e_last);

    BPE_STAMP(2);
    // ---- 3. word-table probe per piece ----------------------------------------
    lds_u16 *stage = (lds_u16 *)s_stage;
    lds_u8 *cnt = (lds_u8 *)s_cnt;
    // pieces for the wave BPE: the byte classes are dead now; a miss spans >= 2
    // bytes, so a chunk has at most CHUNK / 2 <= WIN / 2 of them
    uint16_t *s_pend = reinterpret_cast<uint16_t *>(s_cls);
    const lds_u32 *w32 = (const lds_u32 *)s_win;
    if (tid == 0) s_scratch[1] = 0;
    __syncthreads();
    for (int pi = tid; pi < np; pi += TOK_THREADS) {
        const uint32_t pc = s_pieces[pi];
        const int prel = (int)(pc & 0xFFFu);
        const int nxt = pi + 1 < np ? (int)(s_pieces[pi + 1] & 0xFFFu) : e_last;
        bool pend = false;
        if (pc & (1u << 12)) {
            const int m = special_match(C, c0 + prel);
            stage[prel] = (uint16_t)T.special_id[m < 0 ? 0 : m];
            cnt[pi] = 1;
        } else if (nxt < 0 || nxt - prel > BPE_MAX_WAVE) {
            // long piece: finished by k_bpe_long
            const uint32_t li = atomicAdd(long_count, 1u);
            if (li < long_cap) {
                long_list[li].pos = (uint64_t)(c0 + prel);
                long_list[li].len = nxt < 0 ? 0u : (uint32_t)(nxt - prel);  // 0: find the end
                long_list[li].chunk = (uint32_t)ci;
                long_list[li].k = 0;
            }
            stage[prel] = (uint16_t)(li & 0xFFFFu);
            stage[prel + 1] = (uint16_t)(li >> 16);
            cnt[pi] = CNT_LONG;  // marker
        } else {
            const int n = nxt - prel;
            if (n <= 16) {
                const int wr = prel + HALO_L;
                const int a = wr >> 2;
                const uint32_t sh = (uint32_t)(wr & 3);
                const uint32_t x0 = w32[a], x1 = w32[a + 1], x2 = w32[a + 2], x3 = w32[a + 3], x4 = w32[a + 4];
                const W16 raw{__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh),
                              __builtin_amdgcn_alignbyte(x3, x2, sh), __builtin_amdgcn_alignbyte(x4, x3, sh)};
                const W16 w = keep_bytes(raw, n);
                const int id = probe_result(probe_load(T, hash16(w, (uint32_t)n, 0u)), (uint32_t)n, w);
                if (id >= 0) {
                    stage[prel] = (uint16_t)id;
                    cnt[pi] = 1;
                } else {
                    pend = true;
                }
            } else {
                // 17..64 bytes: hash the LDS bytes, compare the payload beyond 16 from the pool
                const uint32_t un = (uint32_t)n;
                uint32_t h = hinit(un, 0u);
                W16 first{0, 0, 0, 0};
                for (uint32_t b0 = 0; b0 < un; b0 += 16) {
                    uint32_t c[4] = {0, 0, 0, 0};
                    for (uint32_t k = 0; k < 16 && b0 + k < un; ++k)
                        c[k >> 2] |= (uint32_t)win[prel + HALO_L + b0 + k] << (8 * (k & 3));
                    if (b0 == 0) first = W16{c[0], c[1], c[2], c[3]};
                    h = hmix(hmix(hmix(hmix(h, c[0]), c[1]), c[2]), c[3]);
                }
                const Probe P = probe_load(T, hfinal(h));
                int id = -1;
                for (int which = 0; which < 2 && id < 0; ++which) {
                    const uint4 sa = which ? P.a2 : P.a1, sb = which ? P.b2 : P.b1;
                    if (!slot_match(sa, sb, un, first)) continue;
                    bool ok = true;
                    for (uint32_t k = 16; k < un && ok; ++k) ok = T.vpool[sa.z + k] == win[prel + HALO_L + k];
                    if (ok) id = (int32_t)sa.y;
                }
                if (id >= 0) {
                    stage[prel] = (uint16_t)id;
                    cnt[pi] = 1;
                } else {
                    pend = true;
                }
            }
        }
        const uint64_t pm = __ballot(pend);
        if (pm) {
            const int leader = __builtin_ctzll(pm);
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(&s_scratch[1], (uint32_t)__popcll(pm));
            base = lane_bcast(base, leader);
            if (pend) s_pend[base + __popcll(pm & ((1ull << lane) - 1ull))] = (uint16_t)pi;
        }
    }
    __syncthreads();

    BPE_STAMP(3);
    const int npend = (int)s_scratch[1];
    // ---- 4a. misses of <= LANE_BPE bytes: one word per lane (bpe_lane) ----------
    for (int q0 = 0; q0 < npend; q0 += TOK_THREADS) {  // (wave-uniform)
        const int q = q0 + lane;
        int pi = 0, prel = 0, n = 0;
        if (q < npend) {
            pi = s_pend[q];
            prel = (int)(s_pieces[pi] & 0xFFFu);
            const int nxt = pi + 1 < np ? (int)(s_pieces[pi + 1] & 0xFFFu) : e_last;
            n = nxt - prel;
        }
        const bool mine = n >= 2 && n <= LANE_BPE;
        if (!__any(mine)) continue;
        uint32_t sy[LANE_BPE];
#pragma unroll
        for (int k = 0; k < LANE_BPE; ++k) sy[k] = mine && k < n ? (uint32_t)T.byte_id[win[prel + HALO_L + k]] : 0u;
        const int k_out = bpe_lane(T, sy, mine ? n : 0);
        if (mine) {
#pragma unroll
            for (int k = 0; k < LANE_BPE; ++k)
                if (k < k_out) stage[prel + k] = (uint16_t)sy[k];
            cnt[pi] = (uint8_t)k_out;
        }
    }
    __syncthreads();
    BPE_STAMP(6);
    // ---- 4. wave BPE of the (longer) misses, packed: consecutive misses share the lanes --
    for (int q = 0; q < npend;) {
        int total = 0, nw = 0, wprel = 0, wpi = 0;
        uint32_t sym = 0;
        uint64_t heads = 0;
        while (q < npend) {  // wave-uniform packing (every miss is 2..64 bytes)
            const int pi = s_pend[q];
            const int prel = (int)(s_pieces[pi] & 0xFFFu);
            const int nxt = pi + 1 < np ? (int)(s_pieces[pi + 1] & 0xFFFu) : e_last;
            const int n = nxt - prel;
            if (n <= LANE_BPE) {  // (done in 4a)
                ++q;
                continue;
            }
            if (total + n > 64) break;
            if (lane >= total && lane < total + n) sym = (uint32_t)T.byte_id[win[prel + HALO_L + lane - total]];
            if (lane == nw) {
                wprel = prel;
                wpi = pi;
            }
            heads |= 1ull << total;
            total += n;
            ++nw;
            ++q;
        }
        if (total == 0) continue;  // (only short misses were left: 4a took them)
        const int k = bpe_wave_seg(T, sym, total, heads, (lds_u32 *)s_tmp, (lds_u32 *)s_tmpv);
        const uint64_t upto = lane == 63 ? heads : heads & ((2ull << lane) - 1ull);
        const int seg = __popcll(upto) - 1;
        const int start = upto ? 63 - __builtin_clzll(upto) : 0;
        const int sprel = __shfl(wprel, seg < 0 ? 0 : seg, 64);
        const int spi = __shfl(wpi, seg < 0 ? 0 : seg, 64);
        if (lane < k) {
            stage[sprel + lane - start] = (uint16_t)sym;
            const bool lastl = lane == k - 1 || ((heads >> (lane + 1)) & 1ull);
            if (lastl) cnt[spi] = (uint8_t)(lane - start + 1);
        }
        __syncthreads();
    }

    BPE_STAMP(4);
    // ---- 5. compact ids into this chunk's tokc slice ------------------------------
    const int per = (np + TOK_THREADS - 1) / TOK_THREADS;
    const int a0 = tid * per < np ? tid * per : np;
    const int a1 = a0 + per < np ? a0 + per : np;
    uint32_t mine = 0;
    for (int i = a0; i < a1; ++i) mine += s_cnt[i] == CNT_LONG ? 1u : s_cnt[i];
    uint32_t total;
    const uint32_t base0 = block_excl_sum<TOK_THREADS>(mine, &total, s_scratch + 2);
    uint32_t *dst = tokc + ci * STAGE;
    uint32_t base = base0;
    // the list is packed in LDS first (window and classes are dead now) and
    // written as whole 16-B lanes: scattered 4-B non-temporal stores cost ~3.5x
    // the list's bytes in HBM writes
    const bool packed = total <= (uint32_t)(2 * WIN / 4);
    lds_u32 *pk = (lds_u32 *)s_wc;
    for (int i = a0; i < a1; ++i) {
        const int prel = s_pieces[i] & 0xFFF;
        const int k = s_cnt[i];
        if (k == CNT_LONG) {
            const uint32_t mark = LONG_MARK | (uint32_t)s_stage[prel] | ((uint32_t)s_stage[prel + 1] << 16);
            if (packed) pk[base] = mark;
            else dst[base] = mark;
            ++base;
            continue;
        }
        if (packed) {
            for (int j = 0; j < k; ++j) pk[base + j] = (uint32_t)s_stage[prel + j];
        } else {
            for (int j = 0; j < k; ++j) __builtin_nontemporal_store((uint32_t)s_stage[prel + j], dst + base + j);
        }
        base += k;
    }
    __syncthreads();
    if (packed) {
        for (uint32_t e = 4u * (uint32_t)tid; e < total; e += 4u * TOK_THREADS) {
            u32x4 v;
            v.x = pk[e];
            v.y = pk[e + 1];
            v.z = pk[e + 2];
            v.w = pk[e + 3];
            __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(dst + e));
        }
    }
    // the stage is free now: it holds each piece's entry offset in the chunk
    uint16_t *s_poff = s_stage;
    base = base0;
    for (int i = a0; i < a1; ++i) {
        s_poff[i] = (uint16_t)base;
        base += s_cnt[i] == CNT_LONG ? 1u : s_cnt[i];
    }
    __syncthreads();
    BPE_STAMP(5);
    if (tid == 0) chunk_cnt[ci] = chunk_ent[ci] = total;
    // record boundaries owned by this chunk: local entry offset of the first
    // piece at or after the boundary (k_bpe_long adds long pieces' extra ids)
    const int k_lo = (int)(r_lo - ra);
    for (int k = k_lo + tid; k < nrb; k += TOK_THREADS) {
        const int64_t pos = (int64_t)off[ra + k];
        if (pos >= c1) break;
        const int rel = (int)(pos - c0);
        int lo = 0, hi = np;
        while (lo < hi) {
            const int m = (lo + hi) >> 1;
            if ((int)(s_pieces[m] & 0xFFF) < rel) lo = m + 1; else hi = m;
        }
        rec_local[ra + k] = lo < np ? (uint32_t)s_poff[lo] : total;
    }
}

// ---------------------------------------------------------------------------
// Long pieces (> 64 bytes, or running past their chunk's window): one wave
// each, symbols in `scratch` at the piece's own byte positions (u16), the same
// merge steps as bpe_wave in 64-symbol tiles.  The ids stay in `scratch`;
// the chunk's count and the local offsets of its later records grow by k - 1.
// (r04) A piece of <= LONG_LDS symbols runs in LDS with every pair's merge value cached: a merge
// step reads the cached ranks for its minimum and its candidates, carries the values of pairs no
// merge touched through the compaction, and probes the merge table only for the pairs next to a
// merged symbol -- O(merges) probes per step instead of O(symbols) twice.  Longer pieces use the
// global scratch as before.
constexpr int LONG_LDS = 1024;
__global__ __launch_bounds__(64) void k_bpe_long(DevTok T, const uint8_t *__restrict__ text, int64_t N,
                                                 const uint64_t *__restrict__ off, int64_t R,
                                                 const uint32_t *__restrict__ long_count, BpeLong *__restrict__ list,
                                                 uint32_t long_cap, uint16_t *__restrict__ scratch,
                                                 uint32_t *__restrict__ chunk_cnt, uint32_t *__restrict__ rec_local,
                                                 uint32_t *__restrict__ err) {
    __shared__ uint16_t s_sym[LONG_LDS + 64];
    __shared__ uint32_t s_val[LONG_LDS + 64];  // merge_val of pair (j, j + 1); NOVAL: not known
    __shared__ uint16_t s_byte_id[256];
    uint32_t n_long = *long_count;
    if (n_long > long_cap) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(err, 1u);
        n_long = long_cap;
    }
    if (blockIdx.x >= n_long) return;  // (the grid is sized for the held-out corpus; most texts have few)
    for (int i = threadIdx.x; i < 256; i += 64) s_byte_id[i] = T.byte_id[i];
    __syncthreads();
    const Ctx C{&T, nullptr, nullptr, INT64_MIN / 4, text, N, off, R};  // no window: global reads
    const int lane = lane_id();
    const uint64_t lt = (1ull << lane) - 1ull;
    // pieces are taken from a shared cursor (long_count[1]): their lengths vary a lot, and a
    // static stride left waves idle behind the longest
    uint32_t *cursor = const_cast<uint32_t *>(long_count) + 1;
    auto next_piece = [&]() -> uint32_t {
        uint32_t v = 0;
        if (lane == 0) v = atomicAdd(cursor, 1u) + gridDim.x;
        return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
    };
    for (uint32_t li = blockIdx.x; li < n_long; li = next_piece()) {
        const int64_t p = (int64_t)list[li].pos;
        int64_t n = list[li].len;
        // record containing p (its end bounds the piece)
        int64_t lo = 0, hi = R;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if ((int64_t)off[mid + 1] <= p) lo = mid + 1; else hi = mid;
        }
        const int64_t rec = lo;
        if (n == 0) n = bpe_piece_end(C, p) - p;  // ran past its chunk's window
        int64_t m = n;
        if (n <= LONG_LDS) {
            // not known: merged / right neighbour changed (NOVAL), left neighbour of a merge (NOVAL2);
            // merge_val's "no merge" is 0xFFFFFFFF, its ranks stay below 0xFFFD
            constexpr uint32_t NOVAL = 0xFFFFFFFEu, NOVAL2 = 0xFFFFFFFDu;
            const int nn = (int)n;
            for (int j = lane; j < nn; j += 64) s_sym[j] = s_byte_id[text[p + j]];
            __syncthreads();
            for (int j = lane; j + 1 < nn; j += 64) s_val[j] = merge_val(T, s_sym[j], s_sym[j + 1]);
            __syncthreads();
            int mm = nn;
            for (;;) {
                uint32_t rmin = 0xFFFFu;
                for (int j = lane; j + 1 < mm; j += 64) {
                    const uint32_t r = s_val[j] >> 16;
                    rmin = r < rmin ? r : rmin;
                }
                rmin = wave_min_u32(rmin);
                if (rmin == 0xFFFFu) break;
                // merge its occurrences left to right, compact in place; a kept symbol keeps its
                // pair's value when neither it nor its right neighbour changes
                bool blocked = false;
                int outp = 0;
                for (int t0 = 0; t0 < mm; t0 += 64) {
                    const int j = t0 + lane;
                    const uint32_t sym = j < mm ? s_sym[j] : 0u;
                    const uint32_t v = j + 1 < mm ? s_val[j] : 0xFFFFFFFFu;
                    const uint64_t cand = __ballot(j + 1 < mm && (v >> 16) == rmin);
                    const uint64_t sel = leftmost_alternating(cand, blocked);
                    const uint64_t tile = (mm - t0 >= 64) ? ~0ull : ((1ull << (mm - t0)) - 1ull);
                    uint64_t live = tile & ~(sel << 1);
                    if (blocked) live &= ~1ull;
                    const bool me = (sel >> lane) & 1ull;
                    // the right neighbour of a kept symbol changes when it is merged away (my
                    // pair selected) or merges with its own right neighbour (lane + 1 selected)
                    const bool next_sel = lane < 63 ? ((sel >> (lane + 1)) & 1ull) : false;
                    const uint32_t out = me ? (v & 0xFFFFu) : sym;
                    const uint32_t outv = (me || next_sel) ? NOVAL : v;
                    __syncthreads();  // every lane has read its tile before any lane writes
                    if ((live >> lane) & 1ull) {
                        const int o = outp + __popcll(live & lt);
                        s_sym[o] = (uint16_t)out;
                        s_val[o] = outv;
                    }
                    __syncthreads();
                    outp += __popcll(live);
                    blocked = (sel >> 63) & 1ull;
                }
                // (a tile's last kept symbol whose neighbour sat in the next tile, and a merge
                // reaching across a tile edge, leave the value at NOVAL through next_sel / me; a
                // symbol whose left neighbour merged keeps its own pair, which is unchanged)
                mm = outp;
                // the left neighbour of a merged symbol: its pair changed too (the tile's last
                // kept symbol cannot see a merge at the next tile's first pair); runs before the
                // last symbol's value is cleared, which may be the merged one
                for (int j = lane; j + 1 < mm; j += 64) {
                    const uint32_t nx = s_val[j + 1], cur = s_val[j];
                    if (nx == NOVAL && cur != NOVAL && cur != NOVAL2) s_val[j] = NOVAL2;
                }
                __syncthreads();
                if (mm > 0 && lane == 0) s_val[mm - 1] = 0xFFFFFFFFu;  // (no pair past the end)
                __syncthreads();
                for (int j = lane; j + 1 < mm; j += 64) {
                    const uint32_t cur = s_val[j];
                    if (cur == NOVAL || cur == NOVAL2) s_val[j] = merge_val(T, s_sym[j], s_sym[j + 1]);
                }
                __syncthreads();
            }
            for (int j = lane; j < mm; j += 64) scratch[p + j] = s_sym[j];
            m = mm;
        } else {
        // initial symbols
        for (int64_t j = lane; j < n; j += 64) scratch[p + j] = s_byte_id[text[p + j]];
        __syncthreads();
        for (;;) {
            // pass 1: lowest rank over all adjacent pairs
            uint32_t rmin = 0xFFFFu;
            for (int64_t j = lane; j + 1 < m; j += 64) {
                const uint32_t v = merge_val(T, scratch[p + j], scratch[p + j + 1]);
                const uint32_t r = v >> 16;
                rmin = r < rmin ? r : rmin;
            }
            rmin = wave_min_u32(rmin);
            if (rmin == 0xFFFFu) break;
            // pass 2: merge its occurrences left to right, compact in place
            bool blocked = false;  // the last pair of the previous tile merged
            int64_t outp = 0;
            for (int64_t t0 = 0; t0 < m; t0 += 64) {
                const int64_t j = t0 + lane;
                const uint32_t sym = j < m ? scratch[p + j] : 0u;
                const uint32_t nx = j + 1 < m ? scratch[p + j + 1] : 0u;
                const uint32_t v = j + 1 < m ? merge_val(T, sym, nx) : 0xFFFFFFFFu;
                const uint64_t cand = __ballot(j + 1 < m && (v >> 16) == rmin);
                const uint64_t sel = leftmost_alternating(cand, blocked);
                const uint64_t tile = (m - t0 >= 64) ? ~0ull : ((1ull << (m - t0)) - 1ull);
                uint64_t live = tile & ~(sel << 1);
                if (blocked) live &= ~1ull;  // removed by the previous tile's last merge
                const bool me = (sel >> lane) & 1ull;
                const uint32_t out = me ? (v & 0xFFFFu) : sym;
                __syncthreads();  // every lane has read its tile before any lane writes
                if ((live >> lane) & 1ull) scratch[p + outp + __popcll(live & lt)] = (uint16_t)out;
                __syncthreads();
                outp += __popcll(live);
                blocked = (sel >> 63) & 1ull;
            }
            m = outp;
            __syncthreads();
        }
        }
        if (lane == 0) {
            list[li].k = (uint32_t)m;
            list[li].len = (uint32_t)n;
            const uint32_t extra = (uint32_t)m - 1u;
            if (extra) {
                atomicAdd(&chunk_cnt[list[li].chunk], extra);
                // later record starts in the same chunk
                const int64_t cend = ((int64_t)list[li].chunk + 1) * CHUNK;
                for (int64_t r = rec + 1; r < R && (int64_t)off[r] < cend; ++r) {
                    if ((int64_t)off[r] > p) atomicAdd(&rec_local[r], extra);
                }
            }
        }
        __syncthreads();
    }
}

hipError_t launch_bpe_chunks(const DevTok &T, const uint8_t *text, int64_t N, const uint64_t *off, int64_t R,
                             const uint32_t *ranges, uint32_t *tokc, uint32_t *chunk_cnt, uint32_t *chunk_ent,
                             uint32_t *rec_local, uint32_t *long_count, BpeLong *long_list, uint32_t long_cap,
                             uint16_t *scratch, uint32_t *err, hipStream_t st) {
    const int64_t n_chunks = (N + CHUNK - 1) / CHUNK;
    if (n_chunks == 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(long_count, 0, 2 * sizeof(uint32_t), st);  // count, k_bpe_long's cursor
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_bpe_chunks, dim3((unsigned)n_chunks), dim3(TOK_THREADS), 0, st, T, text, N, off, R, ranges,
                       tokc, chunk_cnt, chunk_ent, rec_local, long_count, long_list, long_cap);
    // one wave per long piece: the merges of one piece are a dependent chain of L2 round trips,
    // so the pieces in flight are what it runs on (r04: 1024 waves, one per SIMD, was 1.70 ms on
    // the held-out corpus); a block finds no piece and exits at once when there are fewer
constexpr int BPE_LONG_GRID = 2048;
    const int64_t grid = std::min<int64_t>((int64_t)long_cap, BPE_LONG_GRID);
    if (grid > 0)
        hipLaunchKernelGGL(k_bpe_long, dim3((unsigned)grid), dim3(64), 0, st, T, text, N, off, R, long_count, long_list,
                           long_cap, scratch, chunk_cnt, rec_local, err);
    return hipGetLastError();
}

}  // namespace sdl
