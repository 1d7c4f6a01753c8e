// tokenize_unigram.hip -- t5-small tokenization (Precompiled + WhitespaceSplit
// + Metaspace + Unigram) of a text arena on gfx950.
//
// Restates, for a whole arena of records at once, what the reference does one
// record at a time for task=span (TokenizerHolder::get_ids ->
// tokenizers::Tokenizer::encode, rust/src/tokenizer/tokenizer_holder.rs:19-28;
// crate tokenizers 0.13.1) with the t5-small tokenizer.json:
//   AddedVocabulary split (<pad> </s> <unk> <extra_id_k> on the raw text)
//   -> Precompiled normalizer (grapheme clusters + charsmap trie)
//   -> WhitespaceSplit -> Metaspace("▁", prefix) -> Unigram Viterbi.
// The wrapper's </s> ... </s> framing is added at row assembly (pipeline.hip).
//
// One wave64 per 1 KiB chunk (as the other tokenizers).  Raw words -- runs
// between ASCII whitespace, record edges and added tokens -- normalize
// independently (host-checked charsmap facts), so each is settled
// in the chunk:
//   - simple words (printable ASCII, <= UNI_WMAX bytes) are their own
//     normalization: one probe of the word table (vocab "▁w" pieces with their
//     precomputed Viterbi ids) settles most of them;
//   - medium words (other bytes, <= UNI_WMAX) are normalized into an LDS arena
//     through the per-code-point table (one load per char; the trie only for
//     multi-char clusters that start a longer key), then whitespace/"▁" split;
//   - word-table misses and medium pieces go through the Viterbi in two
//     batched phases: every candidate substring of every pending piece of the
//     chunk is one independent cuckoo probe (lanes x 4 in flight), its id and
//     f32 score kept in LDS; then a lane per word runs the DP from LDS only.
// Longer words (or words running past the window) are *long items*: their
// chunk entry is a marker, k_unigram_long finishes them lane per item from a
// global list, ids into a pool the compaction expands; items whose normalized
// text exceeds a lane's scratch go to k_unigram_huge (one wave each).
#include <cstdio>
#include <type_traits>

#include "common.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "tok_device.hpp"
#include "unigram.hpp"

namespace sdl {

namespace {

// (one bit per class: the starts and word ends are found byte-parallel)
enum : uint8_t { U_WS = 1, U_P = 2, U_X = 4, U_SPEC = 8, U_SPX = 16 };
constexpr uint32_t LMARK = 0x80000000u;
// byte x (< 3) of "▁" (U+2581) -- arithmetic, not a global table: a load here
// would make the DP wait for every probe in flight (vmcnt counts in order)
__device__ __forceinline__ uint32_t meta_byte(int x) { return x == 0 ? 0xE2u : x == 1 ? 0x96u : 0x81u; }

// LDS budget: 3 one-wave blocks per SIMD (<= 13.3 KB each) -- the kernel waits
// on probe latency, so resident waves are what it runs on
constexpr int ARENA = 768;  // LDS bytes for normalized medium words
constexpr int WIN_PAD = WIN + 32;   // window + gather padding; the arena follows
constexpr int VP_CAP = UNI_VPC;  // Viterbi jobs per chunk (more: long items)
constexpr int MED_CAP = 128;  // medium words per chunk (more: long items)
constexpr int UNI_WT_UNROLL = 2;  // word-table probes in flight per lane
constexpr uint8_t CNT_LONG = 0xFF;  // s_cnt of a long item
// s_cnt of a piece handed to k_unigram_viterbi: CNT_JOB | its jobs (<= 0x3F), or, a word past UNI_WMAX
// bytes (one job), CNT_JOB | CNT_WIDE | its payload units; the low 6 bits are the payload units either way
constexpr uint8_t CNT_JOB = 0x80, CNT_WIDE = 0x40;
// k_unigram_viterbi: a pass takes the chunk's next jobs whose candidates fit VTCAP (one job
// always does: vp_tasks(UNI_WMAX) = 17 + 16 * 16 < VTCAP) and at most VJP of them (a DP lane each)
constexpr int VJP = 64, VTCAP = 768, VU = 2;  // VU: probes in flight per lane
constexpr int PFX_JOBS = 6;                    // jobs a wide pass takes at most (their prefix bounds in LDS)
static_assert(VJP <= 64 && VTCAP % (64 * VU) == 0 && VTCAP < 0x7FF, "a hit index fits a back pointer's 11 bits");

typedef __attribute__((address_space(3))) double lds_f64;

__device__ __forceinline__ uint32_t uni_ascii(uint32_t b) {
    if (b == 32u || b == 9u || b == 10u || b == 12u || b == 13u) return U_WS;
    if (b - 0x21u < 0x5Eu) return U_P;
    return U_X;
}
// uni_ascii of 4 bytes
__device__ __forceinline__ uint32_t uni_ascii4(uint32_t x) {
    const uint32_t lo7 = ~x & B7, a = x & 0x7F7F7F7Fu;
    const uint32_t ws = (in7(a, 9, 10) | in7(a, 12, 13) | in7(a, 32, 32)) & lo7;
    const uint32_t p = in7(a, 0x21, 0x7E) & lo7;
    return (ws >> 7) | (p >> 6) | ((B7 & ~ws & ~p) >> 5);
}
__device__ __forceinline__ bool ascii_ws(uint32_t b) { return b == 32u || b == 9u || b == 10u || b == 12u || b == 13u; }

__device__ __forceinline__ uint2 cp_ent(const DevTok &T, uint32_t cp) {
    if (cp < 0x10000u) return T.cbmp[cp];
    if (cp >= 0x110000u) cp = 0xFFFDu;
    return T.cent[(uint32_t)T.cpage[cp >> 8] * 256u + (cp & 255u)];
}

// both cuckoo slots of hash h in the word table (UC_WORD keys)
__device__ __forceinline__ Probe probe_load_words(const DevTok &T, uint32_t h) {
    const uint4 *e1 = reinterpret_cast<const uint4 *>(T.wslots + cuckoo_slot1(h, T.wslot_mask));
    const uint4 *e2 = reinterpret_cast<const uint4 *>(T.wslots + cuckoo_slot2(h, T.wslot_mask));
    return Probe{e1[0], e1[1], e2[0], e2[1]};
}

// id of the slot (payload bytes acc(start .. start+n), cont) or -1: exact
template <class Acc>
__device__ int probe_acc(const DevTok &T, const Acc &acc, int start, int n, uint32_t cont, uint32_t *w3 = nullptr) {
    uint32_t h = hinit((uint32_t)n, cont);
    W16 first{0, 0, 0, 0};
    int b0 = 0;
    do {
        W16 c{0, 0, 0, 0};
        for (int k = 0; k < 16 && b0 + k < n; ++k) w16_put(c, k, acc(start + b0 + k));
        if (b0 == 0) first = c;
        h = hmix(hmix(hmix(hmix(h, c.x), c.y), c.z), c.w);
        b0 += 16;
    } while (b0 < n);
    h = hfinal(h);
    const uint32_t key = (uint32_t)n | (cont << 8);
    const Probe P = cont == UC_WORD ? probe_load_words(T, h) : probe_load(T, h);
    for (int which = 0; which < 2; ++which) {
        const uint4 a = which ? P.a2 : P.a1, b = which ? P.b2 : P.b1;
        if (!slot_match(a, b, key, first)) continue;
        bool ok = true;
        for (int k = 16; k < n && ok; ++k) ok = T.vpool[a.z + k] == acc(start + k);
        if (ok) {
            if (w3) *w3 = a.w;
            return (int32_t)a.y;
        }
    }
    return -1;
}

// probe_result that also returns the slot's word 3 (a Unigram piece's f32 score)
__device__ __forceinline__ int probe_result_w3(const Probe &P, uint32_t key, const W16 &c, uint32_t *w3) {
    if (slot_match(P.a1, P.b1, key, c)) { *w3 = P.a1.w; return (int32_t)P.a1.y; }
    if (slot_match(P.a2, P.b2, key, c)) { *w3 = P.a2.w; return (int32_t)P.a2.y; }
    return -1;
}

// The score tokenizers holds for a piece is serde_json's f64 parse of the
// tokenizer.json number (json.hpp): the f32 score or one f64 ulp off it.  The
// device pieces table (sdl_batcher.cpp) marks a piece one ulp off with bit 15
// of its id and gives the direction by the sign of the f32 in word 3 (scores
// are negative log-probabilities: stored as is, one ulp further from zero;
// negated, one ulp nearer); LDS keeps the 16-bit id and the f32 as before.
constexpr uint32_t UNI_ID_MASK = 0x7FFFu;
__device__ __forceinline__ double uni_score64(float f, uint32_t id16) {
    double d = (double)f;
    if (id16 & 0x8000u) {
        const long long b = __double_as_longlong(f < 0.0f ? d : -d);
        d = __longlong_as_double(f < 0.0f ? b + 1 : b - 1);
    }
    return d;
}
__device__ __forceinline__ int uni_piece_id(int y) { return y < 0 ? y : (int)((uint32_t)y & UNI_ID_MASK); }

// Lane I of every 16-lane row's f64, to the whole row (DPP row_newbcast: in the VALU, no LDS).
template <int I>
__device__ __forceinline__ double row_bcast_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x150 + I, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x150 + I, 0xF, 0xF, false);
    return __longlong_as_double((long long)((uint64_t)(uint32_t)hi << 32 | (uint32_t)lo));
}

// Added token "<...>" starting at p: the bytes up to the first '>' (within
// max_special_len, not crossing a boundary) probed as UC_ADDED.  Returns the id
// and its length, or -1.  byte(q) / bnd(q) = byte / "a record starts at q".
template <class Byte, class Bnd>
__device__ int uni_special(const DevTok &T, int64_t p, int64_t N, const Byte &byte, const Bnd &bnd, int *len) {
    for (int k = 1; k < T.max_special_len && p + k < N; ++k) {
        if (bnd(p + k)) return -1;
        if (byte(p + k) == (uint32_t)'>') {
            const int id = probe_acc(T, [&](int i) -> uint32_t { return byte(p + i); }, 0, k + 1, UC_ADDED);
            if (id >= 0) *len = k + 1;
            return id;
        }
    }
    return -1;
}

// Strict UTF-8 decode as oracle/orc_unigram.c (u8len): raw length consumed,
// cp, the sanitized bytes (invalid -> U+FFFD) and their count.
template <class RB>
__device__ __forceinline__ int dec_char(const RB &rb, int64_t q, int64_t end, uint32_t *cp, uint32_t *bytes,
                                        int *blen) {
    const uint32_t b = rb(q);
    if (b < 0x80u) {
        *cp = b;
        *bytes = b;
        *blen = 1;
        return 1;
    }
    int len = 0;
    uint32_t c = 0, mn = 0;
    if ((b & 0xE0u) == 0xC0u) { len = 2; c = b & 0x1Fu; mn = 0x80u; }
    else if ((b & 0xF0u) == 0xE0u) { len = 3; c = b & 0x0Fu; mn = 0x800u; }
    else if ((b & 0xF8u) == 0xF0u) { len = 4; c = b & 0x07u; mn = 0x10000u; }
    bool ok = len > 0 && q + len <= end;
    uint32_t raw = b;
    for (int k = 1; ok && k < len; ++k) {
        const uint32_t x = rb(q + k);
        if ((x & 0xC0u) != 0x80u) ok = false;
        c = c << 6 | (x & 0x3Fu);
        raw |= x << (8 * k);
    }
    if (ok && (c < mn || c > 0x10FFFFu || (c >= 0xD800u && c <= 0xDFFFu))) ok = false;
    if (!ok) {
        *cp = 0xFFFDu;
        *bytes = 0xBDBFEFu;
        *blen = 3;
        return 1;
    }
    *cp = c;
    *bytes = raw;
    *blen = len;
    return len;
}

// Precompiled::normalize of raw word [a, b) (rb = raw bytes); put(byte)
// returns false when the output is full.  ctx_space: the byte before a is ' '
// (a cluster may run on from it; such chars are looked up one by one, as the
// whole cluster -- starting with ' ' -- matches no key).  Per cluster:
//   one char: its own entry (key -> normalization, else kept);
//   more chars, < 6 bytes: the shortest key prefix of the cluster -- the first
//     char itself when it is a key (the rest is dropped), a trie walk when it
//     only starts longer keys, else none -> per char;
//   otherwise per char.
template <class RB, class Put>
__device__ bool normalize_span(const DevTok &T, const RB &rb, int64_t a, int64_t b, bool ctx_space, const Put &put) {
    GState g;
    gstate_reset(g);
    if (ctx_space) gcb_break(g, uni_ascii_props(0x20u));
    auto put_entry = [&](uint2 e, uint32_t bytes, int bl) -> bool {
        if (!(e.x & CP_KEY)) {
            for (int k = 0; k < bl; ++k)
                if (!put((bytes >> (8 * k)) & 0xFFu)) return false;
            return true;
        }
        if (e.x & CP_INLINE) {
            const int nb = (int)((e.x >> 11) & 7u);
            for (int k = 0; k < nb; ++k)
                if (!put((e.y >> (8 * k)) & 0xFFu)) return false;
            return true;
        }
        for (uint32_t i = e.y; i < T.tnorm_len && T.tnorm[i]; ++i)
            if (!put(T.tnorm[i])) return false;
        return true;
    };
    bool first = true;
    int64_t q = a;
    // the entry of the char that ended the last cluster (its load is reused as
    // the next cluster's first: the chain of dependent loads is one per non-ASCII
    // char, and ASCII chars only need their property byte -- uni_ascii_props)
    uint32_t c_cp = 0xFFFFFFFFu;
    uint2 c_e = make_uint2(0u, 0u);
    while (q < b) {
        const int64_t cs = q;
        {  // printable ASCII followed by ASCII (or the end): a one-char cluster of
           // GCB Other that the charsmap keeps (both host-checked): no table load
            const uint32_t c = rb(q);
            if (c - 0x21u < 0x5Eu && (q + 1 >= b || rb(q + 1) < 0x80u)) {
                gcb_break(g, 0u);
                first = false;
                if (!put(c)) return false;
                ++q;
                continue;
            }
        }
        uint32_t cp0, by0;
        int bl0;
        q += dec_char(rb, q, b, &cp0, &by0, &bl0);
        const uint2 e0 = cp0 == c_cp ? c_e : cp_ent(T, cp0);
        const bool brk = gcb_break(g, e0.x & 0xFFu);
        const bool forced = first && ctx_space && !brk;
        first = false;
        uint32_t buf0 = by0, buf1 = 0;  // the cluster's first 8 sanitized bytes
        int L = bl0, nch = 1;
        while (q < b) {
            uint32_t cp2, by2;
            int bl2;
            const int rl = dec_char(rb, q, b, &cp2, &by2, &bl2);
            uint32_t pr2;
            if (cp2 < 0x80u) {
                pr2 = uni_ascii_props(cp2);
            } else {
                c_e = cp_ent(T, cp2);
                c_cp = cp2;
                pr2 = c_e.x & 0xFFu;
            }
            GState g2 = g;
            if (gcb_break(g2, pr2)) break;
            g = g2;
            for (int k = 0; k < bl2; ++k, ++L) {
                const uint32_t v = (by2 >> (8 * k)) & 0xFFu;
                if (L < 4) buf0 |= v << (8 * L);
                else if (L < 8) buf1 |= v << (8 * (L - 4));
            }
            ++nch;
            q += rl;
        }
        if (nch == 1) {
            if (!put_entry(e0, by0, bl0)) return false;
            continue;
        }
        if (!forced && L < 6) {
            if (e0.x & CP_KEY) {  // the shortest key prefix is the first char: the rest is dropped
                if (!put_entry(e0, by0, bl0)) return false;
                continue;
            }
            if (e0.x & CP_PREFIX) {
                const int32_t r = trie_shortest(T.trie, T.trie_units, [&](int i) -> uint32_t {
                    return i < 4 ? (buf0 >> (8 * i)) & 0xFFu : (buf1 >> (8 * (i - 4))) & 0xFFu;
                }, L);
                if (r >= 0) {
                    bool ok = true;
                    for (uint32_t i = (uint32_t)r; ok && i < T.tnorm_len && T.tnorm[i]; ++i) ok = put(T.tnorm[i]);
                    if (!ok) return false;
                    continue;
                }
            }
        }
        for (int64_t x = cs; x < q;) {  // per char
            uint32_t c3, b3;
            int l3;
            x += dec_char(rb, x, b, &c3, &b3, &l3);
            if (!put_entry(cp_ent(T, c3), b3, l3)) return false;
        }
    }
    return true;
}

// White_Space of the normalized char at nb(i); *len = its byte length
template <class NB>
__device__ __forceinline__ bool norm_ws(const DevTok &T, const NB &nb, int i, int *len) {
    const uint32_t b = nb(i);
    if (b < 0x80u) {
        *len = 1;
        return ascii_ws(b) || b == 0x0Bu;
    }
    const int l = u8len_lead(b);
    uint32_t cp = b & (l == 2 ? 0x1Fu : l == 3 ? 0x0Fu : 0x07u);
    for (int j = 1; j < l; ++j) cp = cp << 6 | (nb(i + j) & 0x3Fu);
    *len = l;
    return uni_white_space(cp);  // (host-checked against the table's GP_WS bits)
}

// ---- long items: global scratch, one lane, sequential -------------------------
struct Scratch {
    uint8_t *nb;     // normalized bytes
    UniNode *nodes;  // Viterbi nodes
    uint32_t *ids;   // ids of the item
    int cap;         // normalized byte capacity (ids: 2 * cap + 8, nodes: cap + 8)
};

struct GNodes {
    UniNode *v;
    __device__ void set(int i, double s, int st, int id) const { v[i] = UniNode{s, st, id}; }
    __device__ double score(int i) const { return v[i].score; }
    __device__ int start(int i) const { return v[i].start; }
    __device__ int id(int i) const { return v[i].id; }
};

// WhitespaceSplit + Metaspace + Unigram over S.nb[0, nl) -> S.ids.  Returns the
// id count, -1 if it exceeds the ids' capacity.
__device__ int tokenize_normalized(const DevTok &T, const Scratch &S, int nl) {
    const uint8_t *nb = S.nb;
    auto nbr = [&](int i) -> uint32_t { return nb[i]; };
    int k = 0;
    const int idcap = 2 * S.cap + 8;
    int i = 0;
    while (i < nl) {
        int l;
        if (norm_ws(T, nbr, i, &l)) { i += l; continue; }
        int j = i;
        while (j < nl && !norm_ws(T, nbr, j, &l)) j += l;
        // word [i, j): pieces before every "▁"; a word not starting with one gets one
        int ps = i;
        bool virt = !(j - i >= 3 && nb[i] == 0xE2 && nb[i + 1] == 0x96 && nb[i + 2] == 0x81);
        for (int t = i + 1; t <= j; ++t) {
            const bool cut = t == j || (t + 3 <= j && nb[t] == 0xE2 && nb[t + 1] == 0x96 && nb[t + 2] == 0x81);
            if (!cut) continue;
            const int off = virt ? 3 : 0;
            const int n = t - ps + off;
            auto acc = [&](int x) -> uint32_t { return x < off ? meta_byte(x) : nb[ps + x - off]; };
            auto cand = [&](int s, int e, double *sc) -> int {
                int id;
                if (s == 0) id = (e - 3 <= T.maxlen_meta) ? probe_acc(T, acc, 3, e - 3, UC_META) : -1;
                else id = (e - s <= T.maxlen_first) ? probe_acc(T, acc, s, e - s, UC_PIECE) : -1;
                id = uni_piece_id(id);
                if (id >= 0) *sc = T.uscore[id];
                return id;
            };
            if (k + n + 1 > idcap) return -1;
            GNodes nodes{S.nodes};
            const int base = k;
            k += unigram_viterbi(acc, n, cand, nodes, T.unk_score, T.unk_id, T.maxlen_piece,
                                 [&](int x, int id) { S.ids[base + x] = (uint32_t)id; });
            ps = t;
            virt = false;
        }
        i = j;
    }
    return k;
}

// Writes an item's k ids (id(j)) to the pool, points its chunk entry at them
// and shifts the chunk's id count and later record offsets by k - 1.
template <class Id>
__device__ void finalize_item(uint32_t c, uint32_t e, int64_t p, int64_t rec, int k, const Id &id,
                              const uint64_t *off, int64_t R, uint32_t *tokc, uint32_t *chunk_cnt, uint32_t *rec_local,
                              uint32_t *pool, uint32_t *pool_count, uint32_t pool_cap, uint32_t *err) {
    // pool word 0 is an empty item; allocations start at 1
    const uint32_t at = 1u + atomicAdd(pool_count, (uint32_t)k + 1u);
    if ((uint64_t)at + (uint32_t)k + 1u > pool_cap) {
        atomicOr(err, 4u);
        k = 0;
        tokc[(int64_t)c * UNI_STAGE + e] = LMARK;
    } else {
        pool[at] = (uint32_t)k;
        for (int j = 0; j < k; ++j) pool[at + 1 + j] = id(j);
        tokc[(int64_t)c * UNI_STAGE + e] = LMARK | at;
    }
    const uint32_t extra = (uint32_t)k - 1u;  // the entry counted one id
    if (extra) {
        atomicAdd(&chunk_cnt[c], extra);
        const int64_t cend = ((int64_t)c + 1) * CHUNK;
        for (int64_t r = rec + 1; r < R && (int64_t)off[r] < cend; ++r)
            if ((int64_t)off[r] > p) atomicAdd(&rec_local[r], extra);
    }
}

__device__ __forceinline__ int64_t record_of(const uint64_t *off, int64_t R, int64_t p, int64_t lo = 0,
                                             int64_t hi = -1) {
    if (hi < 0) hi = R;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int64_t)off[mid + 1] <= p) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// End of a long item's raw word that ran past its chunk's window.
template <class Byte>
__device__ int64_t word_end_b(const DevTok &T, const Byte &byte, int64_t N, int64_t p, int64_t re) {
    auto bnd = [&](int64_t q) -> bool { return q >= re; };
    int64_t end;
    for (end = p + 1; end < re; ++end) {
        const uint32_t b = byte(end);
        if (ascii_ws(b)) break;
        int l;
        if (b == (uint32_t)'<' && T.n_special && uni_special(T, end, N, byte, bnd, &l) >= 0) break;
    }
    return end;
}
__device__ int64_t word_end(const DevTok &T, const uint8_t *text, int64_t N, int64_t p, int64_t re) {
    return word_end_b(T, [&](int64_t q) -> uint32_t { return text[q]; }, N, p, re);
}

// Finishes long item (chunk c, tokc entry e, raw start p, raw length len or
// 0 = unknown): returns false when its normalized text exceeds S.cap and
// !last_resort (nothing written).
__device__ bool finish_long(const DevTok &T, const uint8_t *text, int64_t N, const uint64_t *off, int64_t R,
                            uint32_t c, uint32_t e, int64_t p, int64_t len, const Scratch &S, uint32_t *tokc,
                            uint32_t *chunk_cnt, uint32_t *rec_local, uint32_t *pool, uint32_t *pool_count,
                            uint32_t pool_cap, uint32_t *err, bool last_resort) {
    const int64_t rec = record_of(off, R, p), rs = (int64_t)off[rec];
    const int64_t re = (int64_t)off[rec + 1] < N ? (int64_t)off[rec + 1] : N;
    auto byte = [&](int64_t q) -> uint32_t { return text[q]; };
    const int64_t end = len ? p + len : word_end(T, text, N, p, re);
    const bool ctx_space = p > rs && text[p - 1] == (uint8_t)' ';
    int nl = 0;
    const bool ok = normalize_span(T, byte, p, end, ctx_space, [&](uint32_t v) -> bool {
        if (nl >= S.cap) return false;
        S.nb[nl++] = (uint8_t)v;
        return true;
    });
    int k = 0;
    if (!ok) {
        if (!last_resort) return false;
        atomicOr(err, 16u);  // a whitespace-free run beyond UNI_HUGE_NORM normalized bytes: dropped
    } else {
        k = tokenize_normalized(T, S, nl);
        if (k < 0) {
            atomicOr(err, 2u);
            k = 0;
        }
    }
    finalize_item(c, e, p, rec, k, [&](int j) { return S.ids[j]; }, off, R, tokc, chunk_cnt, rec_local, pool,
                  pool_count, pool_cap, err);
    return true;
}

// ---- the chunk kernel's batched Viterbi ---------------------------------------
// A Viterbi piece (vp) is "▁" + payload, payload = LDS bytes [src, src + L).
// Its candidates are laid out row by row: the "▁" row (payload prefixes of
// 0..min(L, Mm) bytes), then one row per payload start i (ends i+1 ..
// min(L, i + Mf)).
__host__ __device__ constexpr int vp_c0(int L, int Mm) { return (L < Mm ? L : Mm) + 1; }
__host__ __device__ constexpr int vp_rowoff(int i, int L, int Mf) {  // sum_{k<i} min(L-k, Mf)
    const int K = L > Mf ? L - Mf : 0;
    if (i <= K) return i * Mf;
    return K * Mf + (i - K) * L - (K + i - 1) * (i - K) / 2;
}
__host__ __device__ constexpr int vp_tasks(int L, int Mm, int Mf) { return vp_c0(L, Mm) + vp_rowoff(L, L, Mf); }
// a pass always takes its first job whole: the widest job the chunk kernel hands over (wide_ok:
// maxlen_first < UNI_VRING, maxlen_meta + 3 < UNI_VRING) has its candidates within VTCAP
static_assert(vp_tasks(UNI_VMAX, UNI_VRING - 4, UNI_VRING - 1) <= VTCAP && vp_tasks(UNI_WMAX, UNI_WMAX, UNI_WMAX) <= VTCAP,
              "one job fits a pass");
// local index of candidate (i, j) (i = -1: the "▁" row), or -1 if out of range
__device__ __forceinline__ int vp_local(int i, int j, int L, int Mm, int Mf) {
    if (i < 0) return j <= Mm && j <= L ? j : -1;
    if (j - i > Mf || j > L || j <= i) return -1;
    return vp_c0(L, Mm) + vp_rowoff(i, L, Mf) + (j - i - 1);
}
// inverse of vp_local
__device__ __forceinline__ void vp_decode(int t, int L, int Mm, int Mf, int *i, int *j) {
    const int c0 = vp_c0(L, Mm);
    if (t < c0) { *i = -1; *j = t; return; }
    int r = t - c0;
    const int K = L > Mf ? L - Mf : 0;
    if (r < K * Mf) { *i = r / Mf; *j = *i + 1 + r % Mf; return; }
    r -= K * Mf;
    int row = K;
    while (r >= L - row) { r -= L - row; ++row; }
    *i = row;
    *j = row + 1 + r;
}

// 16 bytes at LDS byte offset b (dword loads + alignbyte), first n kept
__device__ __forceinline__ W16 lds_w16(const lds_u32 *w32, int b, int n) {
    const int a = b >> 2;
    const uint32_t sh = (uint32_t)(b & 3);
    const uint32_t x0 = w32[a], x1 = w32[a + 1], x2 = w32[a + 2], x3 = w32[a + 3], x4 = w32[a + 4];
    const W16 raw{__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh),
                  __builtin_amdgcn_alignbyte(x3, x2, sh), __builtin_amdgcn_alignbyte(x4, x3, sh)};
    return keep_bytes(raw, n);
}

}  // namespace

// Diagnostic build (-DSDL_STAMPS): lane 0 of every block adds the s_memtime
// cycles between phase boundaries into sdl_uni_cycles[]; never in the product.
#ifdef SDL_STAMPS
__device__ unsigned long long sdl_uni_cycles[8];
#define UNI_STAMP(k)                                                                  \
    do {                                                                              \
        if (threadIdx.x == 0) {                                                       \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();              \
            atomicAdd(&sdl_uni_cycles[k], t_ - stamp_prev_);                          \
            stamp_prev_ = t_;                                                         \
        }                                                                             \
    } while (0)
// counts (stamps build): 0 chunks 1 pieces 2 Viterbi jobs 3 their candidates 4 Viterbi passes 5 hits
// 6 medium words
__device__ unsigned long long sdl_uni_counts[32];
#define UNI_COUNT(k, v) do { atomicAdd(&sdl_uni_counts[k], (unsigned long long)(v)); } while (0)
void print_uni_cycles() {
    unsigned long long cn[32];
    if (hipMemcpyFromSymbol(cn, HIP_SYMBOL(sdl_uni_counts), sizeof(cn)) == hipSuccess && cn[0]) {
        fprintf(stderr, "[uni counts] chunks %llu pieces/chunk %.1f jobs/chunk %.2f tasks/chunk %.1f "
                        "viterbi passes/chunk %.2f hits/chunk %.1f medium/chunk %.2f\n", cn[0], (double)cn[1] / cn[0],
                (double)cn[2] / cn[0], (double)cn[3] / cn[0], (double)cn[4] / cn[0], (double)cn[5] / cn[0],
                (double)cn[6] / cn[0]);
    }
    unsigned long long h[8];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(sdl_uni_cycles), sizeof(h)) != hipSuccess) return;
    static const char *names[] = {"", "load+classify+specials", "piece starts", "word table+medium", "-",
                                  "compact+jobs+rec_local", "-", "-"};
    unsigned long long tot = 0;
    for (int i = 1; i < 8; ++i) tot += h[i];
    for (int i = 1; i < 8; ++i)
        fprintf(stderr, "[uni stamps] %-24s %6.2f%%\n", names[i], tot ? 100.0 * (double)h[i] / (double)tot : 0.0);
}
__device__ unsigned long long sdl_vit_cycles[8];
#define VIT_STAMP(k)                                                                  \
    do {                                                                              \
        if (threadIdx.x == 0) {                                                       \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();              \
            atomicAdd(&sdl_vit_cycles[k], t_ - vstamp_);                              \
            vstamp_ = t_;                                                             \
        }                                                                             \
    } while (0)
void print_vit_cycles() {
    unsigned long long h[8];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(sdl_vit_cycles), sizeof(h)) != hipSuccess) return;
    static const char *names[] = {"", "jobs load+task bases", "candidate probes", "DP", "backtrack+write",
                                  "count fixups", "-", "-"};
    unsigned long long tot = 0;
    for (int i = 1; i < 8; ++i) tot += h[i];
    for (int i = 1; i < 6; ++i)
        fprintf(stderr, "[vit stamps] %-24s %6.2f%%\n", names[i], tot ? 100.0 * (double)h[i] / (double)tot : 0.0);
    fprintf(stderr, "[vit stamps] total cycles %llu\n", tot);
}
__device__ unsigned long long sdl_long_cycles[8], sdl_long_counts[4];
#define LONG_STAMP(k)                                                                 \
    do {                                                                              \
        if (threadIdx.x == 0) {                                                       \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();              \
            atomicAdd(&sdl_long_cycles[k], t_ - lstamp_);                             \
            lstamp_ = t_;                                                             \
        }                                                                             \
    } while (0)
#define LONG_COUNT(k, v) do { if (threadIdx.x == 0) atomicAdd(&sdl_long_counts[k], (unsigned long long)(v)); } while (0)
void print_long_cycles() {
    unsigned long long h[8], c[4];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(sdl_long_cycles), sizeof(h)) != hipSuccess) return;
    if (hipMemcpyFromSymbol(c, HIP_SYMBOL(sdl_long_counts), sizeof(c)) != hipSuccess) return;
    static const char *names[] = {"", "load+normalize", "piece select", "probes", "relax", "backtrack", "finalize", "-"};
    unsigned long long tot = 0;
    for (int i = 1; i < 8; ++i) tot += h[i];
    for (int i = 1; i < 7; ++i)
        fprintf(stderr, "[long stamps] %-16s %6.2f%%\n", names[i], tot ? 100.0 * (double)h[i] / (double)tot : 0.0);
    fprintf(stderr, "[long stamps] total cycles %llu items %llu ascii %llu pieces %llu sumL %llu\n", tot, c[0], c[1], c[2],
            c[3]);
}
#else
#define UNI_COUNT(k, v) do {} while (0)
#define UNI_STAMP(k) do {} while (0)
#define VIT_STAMP(k) do {} while (0)
#define LONG_STAMP(k) do {} while (0)
#define LONG_COUNT(k, v) do {} while (0)
#endif

// ---------------------------------------------------------------------------
constexpr int UNI_WAVES = 3;
__global__ __launch_bounds__(TOK_THREADS) __attribute__((amdgpu_waves_per_eu(UNI_WAVES, 8))) void k_unigram_chunks(
    DevTok T, const uint8_t *__restrict__ text, int64_t N, const uint64_t *__restrict__ off, int64_t R,
    const uint32_t *__restrict__ ranges, uint32_t *__restrict__ tokc, uint32_t *__restrict__ chunk_cnt,
    uint32_t *__restrict__ chunk_ent, uint32_t *__restrict__ rec_local, uint32_t *__restrict__ counters,
    uint4 *__restrict__ items, uint32_t item_cap, uint32_t *__restrict__ err) {
    __shared__ __attribute__((aligned(16))) uint8_t s_bytes[WIN_PAD + ARENA + 32];  // window | arena
    constexpr int U_CLS = 0, U_MED = (WIN + 15) & ~15, U_MED_END = U_MED + 2 * MED_CAP;
    __shared__ __attribute__((aligned(16))) uint8_t s_u[U_MED_END];  // classes | medium words
    uint8_t *const s_cls = s_u + U_CLS;
    __shared__ uint32_t s_rbits[RBITS_WORDS + 3];  // (+2: word_len's 64-bit windows)
    __shared__ uint16_t s_pieces[CHUNK + 1];  // prel | SPEC << 12
    // ids staged at their piece's byte offset: a piece may use the bytes up to
    // the next piece (stage_room); one that needs more becomes a long item.  A
    // Viterbi piece's slot holds its first job's index.
    __shared__ uint16_t s_stage[STAGE];
    // ids per piece (<= 2 UNI_WMAX), CNT_LONG = long item, CNT_JOB | n = n Viterbi jobs
    __shared__ uint8_t s_cnt[CHUNK];
    uint16_t *const s_med = (uint16_t *)(s_u + U_MED);  // medium words: piece index | length << 11
    __shared__ uint32_t s_scratch[16];  // 1 jobs 2 arena used 3 medium words; 8.. scan scratch
    __shared__ uint16_t s_vp_src[VP_CAP];  // Viterbi jobs: payload in LDS (window or arena) and length
    __shared__ uint8_t s_vp_len[VP_CAP];

    const int tid = threadIdx.x;
    const int lane = tid;
    const int64_t ci = xcd_chunk();  // this block's chunk
    const int64_t c0 = ci * CHUNK;
    const int64_t c1 = c0 + CHUNK < N ? c0 + CHUNK : N;
    const int64_t w0 = c0 - HALO_L;
    const lds_u8 *win = (const lds_u8 *)s_bytes;
    lds_u8 *bytes = (lds_u8 *)s_bytes;
    lds_u8 *cls = (lds_u8 *)s_cls;
    const lds_u32 *rbits = (const lds_u32 *)s_rbits;
    const lds_u32 *w32 = (const lds_u32 *)s_bytes;
#ifdef SDL_STAMPS
    unsigned long long stamp_prev_ = __builtin_amdgcn_s_memtime();
#endif

    // ---- 1. load + classify ----------------------------------------------------
    const uint4 v = load16(text, c0 + 16 * tid, N);
    *reinterpret_cast<uint4 *>(s_bytes + HALO_L + 16 * tid) = v;
    uint4 hv = make_uint4(0, 0, 0, 0);
    int64_t hp = 0;
    if (tid < (WIN - CHUNK) / 16) {
        hp = tid < HALO_L / 16 ? w0 + 16 * tid : c0 + CHUNK + 16 * (tid - HALO_L / 16);
        hv = load16(text, hp, N);
        *reinterpret_cast<uint4 *>(s_bytes + (hp - w0)) = hv;
    }
    if (tid < 2) *reinterpret_cast<uint4 *>(s_bytes + WIN + 16 * tid) = make_uint4(0, 0, 0, 0);
    if (tid <= RBITS_WORDS + 2) s_rbits[tid] = 0;
    const int64_t ra = ranges[3 * ci], rz = ranges[3 * ci + 1], r_lo = ranges[3 * ci + 2];
    const int nrb = (int)(rz - ra);
    if (tid < 8) s_scratch[tid] = 0;  // (1 jobs 2 arena used 3 medium words 4 payload units)
    __syncthreads();
    for (int k = tid; k < nrb; k += TOK_THREADS) {
        const int rel = (int)((int64_t)off[ra + k] - w0);
        atomicOr(&s_rbits[rel >> 5], 1u << (rel & 31));
    }
    auto classify16 = [&](const uint4 &x, int wi0) {
        *reinterpret_cast<uint4 *>(s_cls + wi0) = make_uint4(uni_ascii4(x.x), uni_ascii4(x.y), uni_ascii4(x.z), uni_ascii4(x.w));
    };
    classify16(v, HALO_L + 16 * tid);
    if (tid < (WIN - CHUNK) / 16) classify16(hv, (int)(hp - w0));
    __syncthreads();

    const Ctx C{&T, win, rbits, w0, text, N, off, R};
    auto cbyte = [&](int64_t q) -> uint32_t { return C.byte(q); };
    auto cbnd = [&](int64_t q) -> bool { return C.rstart(q); };
    auto is_rs = [&](int wi) -> bool { return (rbits[wi >> 5] >> (wi & 31)) & 1u; };
    // added tokens (override the classes of their bytes)
    if (T.n_special) {  // openers found in the lane's registers
        auto opens16 = [](const uint4 &x) {
            constexpr uint32_t o4 = (uint32_t)'<' * 0x01010101u;
            return gather16(~nzb(x.x ^ o4), ~nzb(x.y ^ o4), ~nzb(x.z ^ o4), ~nzb(x.w ^ o4));
        };
        auto do_opens = [&](uint32_t m, int wi0) {
            for (; m; m &= m - 1) {
                const int wi = wi0 + __builtin_ctz(m);
                const int64_t p = w0 + wi;
                if (p < 0 || p >= N) continue;
                int l = 0;
                if (uni_special(T, p, N, cbyte, cbnd, &l) < 0) continue;
                cls[wi] = U_SPEC;
                for (int j = 1; j < l && wi + j < WIN; ++j) cls[wi + j] = U_SPX;
            }
        };
        do_opens(opens16(v), HALO_L + 16 * tid);
        if (tid < (WIN - CHUNK) / 16) do_opens(opens16(hv), (int)(hp - w0));
        __syncthreads();
    }

    UNI_STAMP(1);
    // ---- 2. piece starts: added tokens, and the first byte of every word ------
    const int64_t s0 = c0 + 16 * tid;
    const int nown = s0 >= c1 ? 0 : (int)(c1 - s0 < 16 ? c1 - s0 : 16);
    // a word starts at P/X after WS, an added token or a record start;
    // byte-parallel over the lane's class bytes
    uint32_t pmask, smask;
    {
        const int wi0 = HALO_L + 16 * tid;
        const uint4 kc = *reinterpret_cast<const uint4 *>(s_cls + wi0);
        const uint32_t kw[5] = {*reinterpret_cast<const uint32_t *>(s_cls + wi0 - 4), kc.x, kc.y, kc.z, kc.w};
        const uint32_t rs16 = (uint32_t)((((uint64_t)s_rbits[(wi0 >> 5) + 1] << 32) | s_rbits[wi0 >> 5]) >> (wi0 & 31));
        uint32_t st[4], sp[4];
#pragma unroll
        for (int j = 1; j <= 4; ++j) {
            const uint32_t c = kw[j], pc = __builtin_amdgcn_alignbyte(kw[j], kw[j - 1], 3);
            const uint32_t rsq = expand4((rs16 >> (4 * (j - 1))) & 0xFu);
            sp[j - 1] = bit7(c, 3);  // U_SPEC
            st[j - 1] = sp[j - 1] | (nzb(c & 0x06060606u) & (nzb(pc & 0x19191919u) | rsq));
        }
        const uint32_t own = nown >= 16 ? 0xFFFFu : (1u << nown) - 1u;
        pmask = gather16(st[0], st[1], st[2], st[3]) & own;
        smask = gather16(sp[0], sp[1], sp[2], sp[3]);
    }
    uint32_t np_total;
    uint32_t pbase = block_excl_sum<TOK_THREADS>((uint32_t)__builtin_popcount(pmask), &np_total, s_scratch + 8);
    for (uint32_t m = pmask; m;) {
        const int i = __builtin_ctz(m);
        m &= m - 1;
        s_pieces[pbase++] = (uint16_t)((16 * tid + i) | (((smask >> i) & 1u) << 12));
    }
    __syncthreads();
    const int np = (int)np_total;
    UNI_STAMP(2);

    // ---- 3. per piece: added token / word table / medium normalization / long --
    lds_u16 *stage = (lds_u16 *)s_stage;
    lds_u8 *cnt = (lds_u8 *)s_cnt;
    // stage slots of piece pi: up to the next piece's (the last one: the stage's end)
    auto stage_room = [&](int pi) -> int {
        const int prel = (int)(s_pieces[pi] & 0xFFFu);
        return (pi + 1 < np ? (int)(s_pieces[pi + 1] & 0xFFFu) : STAGE) - prel;
    };
    const lds_u32 *cls32 = (const lds_u32 *)s_cls;
    // Length of the raw word starting at window index wi0: 1..UNI_VMAX, 0 when it
    // runs past the window, UNI_VMAX + 1 when longer (its end is found by the
    // long-item kernel); *simple = printable ASCII only.  Its first 20 classes
    // come in 6 independent dword loads, the end is a bit scan; a word with no end
    // among them takes 7 more loads (52 classes).
    auto word_len = [&](int wi0, bool *simple) -> int {
        const int a = wi0 >> 2;
        const uint32_t sh = (uint32_t)(wi0 & 3);
        const int qp = WIN - 8 - wi0;                   // first offset past the window
        const int64_t lim_n = N - (w0 + wi0);           // offsets >= lim_n: past the text
        {
            uint32_t d[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) d[k] = cls32[a + k];
            uint32_t bnd = 0, nonp = 0;  // bit q: class at offset q is a word boundary / not U_P
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                const uint32_t c = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
                bnd |= gather4(nzb(c & 0x09090909u)) << (4 * k);  // U_WS, U_SPEC
                nonp |= gather4(~bit7(c, 1)) << (4 * k);          // not U_P
            }
            const uint64_t rw = ((uint64_t)rbits[(wi0 >> 5) + 1] << 32) | rbits[wi0 >> 5];
            bnd |= (uint32_t)(rw >> (wi0 & 31));            // record starts
            if (lim_n <= (int64_t)UNI_WMAX) bnd |= ~0u << (int)lim_n;
            bnd &= ((2u << UNI_WMAX) - 1u) & ~1u;           // offsets 1 .. UNI_WMAX
            if (bnd) {
                const int qb = __builtin_ctz(bnd);
                if (qp <= qb) return 0;
                *simple = (nonp & ((1u << qb) - 1u)) == 0u;
                return qb;
            }
        }
        uint32_t d[13];
#pragma unroll
        for (int k = 0; k < 13; ++k) d[k] = cls32[a + k];
        uint64_t bnd = 0, nonp = 0;
#pragma unroll
        for (int k = 0; k < 12; ++k) {
            const uint32_t c = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
            bnd |= (uint64_t)gather4(nzb(c & 0x09090909u)) << (4 * k);
            nonp |= (uint64_t)gather4(~bit7(c, 1)) << (4 * k);
        }
        {  // record starts
            const int w = wi0 >> 5, r = wi0 & 31;
            const uint64_t lo = ((uint64_t)rbits[w + 1] << 32) | rbits[w];
            bnd |= r ? lo >> r | (uint64_t)rbits[w + 2] << (64 - r) : lo;
        }
        if (lim_n <= (int64_t)UNI_VMAX) bnd |= ~0ull << lim_n;
        bnd &= ((2ull << UNI_VMAX) - 1u) & ~1ull;       // offsets 1 .. UNI_VMAX
        const int qb = bnd ? __builtin_ctzll(bnd) : UNI_VMAX + 1;
        if (qp <= qb) return 0;
        *simple = qb <= UNI_VMAX && (nonp & ((1ull << qb) - 1u)) == 0u;
        return qb;
    };
    // jobs past UNI_WMAX bytes fit the Viterbi kernel's node ring
    const bool wide_ok = T.maxlen_first < UNI_VRING && T.maxlen_meta + 3 < UNI_VRING;
    // a Viterbi job: its payload in LDS (window or arena) and length; false when the chunk's
    // jobs or payload units are used up (a long item then)
    auto new_job = [&](int src, int len, int nvp, uint32_t *vp0) -> bool {
        const uint32_t units = (uint32_t)(len > 16 ? (len + 15) >> 4 : 1) * (uint32_t)nvp;  // (nvp > 1: medium, <= 16 each)
        const uint32_t vu = atomicAdd(&s_scratch[1], (uint32_t)nvp | units << 16);  // (one LDS atomic: jobs | units)
        const uint32_t v = vu & 0xFFFFu;
        if ((vu >> 16) + units > (uint32_t)UNI_VPC || v + (uint32_t)nvp > (uint32_t)VP_CAP) return false;
        if (src >= 0) {
            s_vp_src[v] = (uint16_t)src;
            s_vp_len[v] = (uint8_t)len;
        }
        *vp0 = v;
        return true;
    };
    for (int p0 = 0; p0 < np; p0 += TOK_THREADS * UNI_WT_UNROLL) {
        // word-table probes of this lane's next UNI_WT_UNROLL pieces, in flight together
        Probe P[UNI_WT_UNROLL];
        W16 W[UNI_WT_UNROLL];
        int len_u[UNI_WT_UNROLL];
        uint32_t kind[UNI_WT_UNROLL];  // 0 none, 1 probe, 2 medium, 3 long
#pragma unroll
        for (int u = 0; u < UNI_WT_UNROLL; ++u) {
            const int pi = p0 + u * TOK_THREADS + tid;
            kind[u] = 0;
            len_u[u] = 0;
            W[u] = W16{0, 0, 0, 0};
            if (pi >= np) continue;
            const uint32_t pc = s_pieces[pi];
            const int prel = (int)(pc & 0xFFFu);
            const int wi0 = HALO_L + prel;
            if (pc & (1u << 12)) {
                int l = 0;
                const int id = uni_special(T, c0 + prel, N, cbyte, cbnd, &l);
                stage[prel] = (uint16_t)(id < 0 ? T.unk_id : id);
                cnt[pi] = 1;
                continue;
            }
            bool simple = false;
            const int len = word_len(wi0, &simple);
            len_u[u] = len;
            if (len > 0 && len <= UNI_WMAX && simple) {
                W[u] = lds_w16(w32, wi0, len);
                P[u] = probe_load_words(T, hash16(W[u], (uint32_t)len, UC_WORD));
                kind[u] = 1;
            } else if (len > 0 && len <= UNI_WMAX) {
                kind[u] = 2;
            } else {  // a printable ASCII word past UNI_WMAX: a (wide) Viterbi job, else a long item
                kind[u] = len > UNI_WMAX && len <= UNI_VMAX && simple && wide_ok ? 4u : 3u;
            }
        }
#pragma unroll
        for (int u = 0; u < UNI_WT_UNROLL; ++u) {
            if (kind[u] == 0) continue;
            const int pi = p0 + u * TOK_THREADS + tid;
            const int prel = (int)(s_pieces[pi] & 0xFFFu);
            const int wi0 = HALO_L + prel;
            const int len = len_u[u];
            const int room = stage_room(pi);
            bool done = false;
            if (kind[u] == 1) {
                const int packed = probe_result(P[u], (uint32_t)len | (UC_WORD << 8), W[u]);
                if (packed >= 0 && (packed >> 24) <= room) {
                    const int k = packed >> 24;
                    const uint32_t x = (uint32_t)packed & 0xFFFFFFu;
                    if (k == 1) stage[prel] = (uint16_t)x;
                    else
                        for (int j = 0; j < k; ++j) stage[prel + j] = T.wres[x + j];
                    cnt[pi] = (uint8_t)k;
                    done = true;
                } else if (packed < 0 && len + 1 <= room) {  // Viterbi yields <= len + 1 ids
                    // miss: one Viterbi piece, the word's bytes in the window
                    uint32_t vp;
                    if (new_job(wi0, len, 1, &vp)) {
                        stage[prel] = (uint16_t)vp;
                        cnt[pi] = CNT_JOB | 1u;
                        done = true;
                    }
                }
            } else if (kind[u] == 4) {
                uint32_t vp;
                if (len + 1 <= room && new_job(wi0, len, 1, &vp)) {
                    stage[prel] = (uint16_t)vp;
                    cnt[pi] = (uint8_t)(CNT_JOB | CNT_WIDE | (uint32_t)((len + 15) >> 4));
                    done = true;
                }
            } else if (kind[u] == 2) {
                // medium word: normalized in the next pass, all lanes at once
                const uint32_t mq = atomicAdd(&s_scratch[3], 1u);
                if (mq < (uint32_t)MED_CAP) {
                    s_med[mq] = (uint16_t)(pi | len << 11);  // (pi < 2^11, len <= UNI_WMAX)
                    cnt[pi] = 0;
                    done = true;
                }
            }
            if (!done) {  // long item: finished by k_unigram_long; its length (0: unknown) in its stage slot
                cnt[pi] = CNT_LONG;
                stage[prel] = (uint16_t)(len <= UNI_VMAX ? len : 0);
            }
        }
    }
    __syncthreads();

    __syncthreads();
    // medium words (non-ASCII or control bytes, <= UNI_WMAX): normalize into the
    // arena (at most UNI_WMAX bytes each), split, list their Viterbi pieces
    const int nmed = (int)(s_scratch[3] < (uint32_t)MED_CAP ? s_scratch[3] : (uint32_t)MED_CAP);
    for (int mq = lane; mq < nmed; mq += 64) {
        const int pi = s_med[mq] & 0x7FF;
        const int prel = (int)(s_pieces[pi] & 0xFFFu);
        const int wi0 = HALO_L + prel;
        const int len = s_med[mq] >> 11;
        bool done = false;
        const uint32_t a = atomicAdd(&s_scratch[2], (uint32_t)UNI_WMAX);
        if (a + UNI_WMAX <= (uint32_t)ARENA) {
            const int abase = WIN_PAD + (int)a;
            const bool ctx_space = !is_rs(wi0) && win[wi0 - 1] == (uint8_t)' ';
            auto rb = [&](int64_t q) -> uint32_t { return win[(int)(q - w0)]; };
            int nl = 0;
            const bool ok = normalize_span(T, rb, w0 + wi0, w0 + wi0 + len, ctx_space, [&](uint32_t x) -> bool {
                if (nl >= UNI_WMAX) return false;
                bytes[abase + nl++] = (uint8_t)x;
                return true;
            });
            if (ok) {
                // WhitespaceSplit + Metaspace: count the pieces and bound the
                // ids (pass 0), then list them (pass 1)
                auto nb = [&](int i) -> uint32_t { return bytes[abase + i]; };
                int nvp = 0, bound = 0;
                uint32_t vp0 = 0;
                bool fits = true;
                for (int pass = 0; pass < 2 && fits; ++pass) {
                    if (pass == 1) {
                        if (nvp == 0) break;
                        if (bound > stage_room(pi) || nvp > 0x3F) { fits = false; break; }
                        if (!new_job(-1, 0, nvp, &vp0)) { fits = false; break; }
                    }
                    int k = 0, i = 0;
                    while (i < nl) {
                        int l;
                        if (norm_ws(T, nb, i, &l)) { i += l; continue; }
                        int j = i;
                        while (j < nl && !norm_ws(T, nb, j, &l)) j += l;
                        int ps = i;
                        bool virt = !(j - i >= 3 && nb(i) == 0xE2 && nb(i + 1) == 0x96 && nb(i + 2) == 0x81);
                        for (int t = i + 1; t <= j; ++t) {
                            const bool cut = t == j || (t + 3 <= j && nb(t) == 0xE2 && nb(t + 1) == 0x96 &&
                                                        nb(t + 2) == 0x81);
                            if (!cut) continue;
                            const int psrc = virt ? ps : ps + 3;  // payload after the "▁"
                            if (pass == 0) {
                                ++nvp;
                                int chars = 0;
                                for (int x = psrc; x < t; ++x) chars += (nb(x) & 0xC0u) != 0x80u;
                                bound += chars + 1;
                            } else {
                                s_vp_src[vp0 + k] = (uint16_t)(abase + psrc);
                                s_vp_len[vp0 + k] = (uint8_t)(t - psrc);
                                ++k;
                            }
                            ps = t;
                            virt = false;
                        }
                        i = j;
                    }
                }
                if (fits && nvp == 0) {  // nothing left after normalization
                    cnt[pi] = 0;
                    done = true;
                } else if (fits) {  // its Viterbi pieces: consecutive jobs vp0 ..
                    stage[prel] = (uint16_t)vp0;
                    cnt[pi] = (uint8_t)(CNT_JOB | (uint32_t)nvp);
                    done = true;
                }
            }
        }
        if (!done) {  // long item: finished by k_unigram_long
            cnt[pi] = CNT_LONG;
            stage[prel] = (uint16_t)len;
        }
    }
    __syncthreads();
    UNI_STAMP(3);
    // ---- 4. compact ids into this chunk's tokc slice; hand the Viterbi pieces to
    //         k_unigram_viterbi; list the long items --------------------------------
    // list entries / Viterbi jobs of a piece (its payload units: c & 0x3F)
    auto ents = [](uint32_t c) -> uint32_t {
        return c == CNT_LONG ? 1u : (c & CNT_JOB) ? ((c & CNT_WIDE) ? 1u : (c & 0x3Fu)) : c;
    };
    auto jobs_of = [](uint32_t c) -> uint32_t { return c != CNT_LONG && (c & CNT_JOB) ? ((c & CNT_WIDE) ? 1u : (c & 0x3Fu)) : 0u; };
    const int per = (np + TOK_THREADS - 1) / TOK_THREADS;
    const int a0 = tid * per < np ? tid * per : np;
    const int a1 = a0 + per < np ? a0 + per : np;
    auto units = [](int L) -> uint32_t { return L > 16 ? (uint32_t)(L + 15) >> 4 : 1u; };  // payload units of a job
    uint32_t mine = 0;  // entries | jobs << 11 | payload units << 19 (one scan)
    for (int i = a0; i < a1; ++i) {
        const uint32_t c = s_cnt[i];
        mine += ents(c) | jobs_of(c) << 11 | (jobs_of(c) ? (c & 0x3Fu) : 0u) << 19;
    }
    uint32_t tot3;
    const uint32_t ex3 = block_excl_sum<TOK_THREADS>(mine, &tot3, s_scratch + 8);
    const uint32_t total = tot3 & 0x7FFu, njobs = (tot3 >> 11) & 0xFFu;
    uint32_t base = ex3 & 0x7FFu, jb = (ex3 >> 11) & 0xFFu, ub = ex3 >> 19;
    uint32_t *dst = tokc + ci * UNI_STAGE;
    const uint32_t base0 = base;
    uint32_t mywide = 0;
    // jobs: payload (<= UNI_VMAX bytes from the window or the arena) and meta = length |
    // stage position of its ids << 6 | list entry << 18; a word's pieces' ids follow each
    // other from its stage slot, each piece bounded by its chars + 1
    for (int i = a0; i < a1; ++i) {
        const uint32_t c = s_cnt[i];
        if (!jobs_of(c)) {
            base += ents(c);
            continue;
        }
        const int prel = s_pieces[i] & 0xFFF;
        const int vp0 = s_stage[prel];
        int pos = prel;
        for (uint32_t q = 0; q < jobs_of(c); ++q, ++base, ++jb) {
            const int L = s_vp_len[vp0 + q], src = s_vp_src[vp0 + q];
            int chars = 0;
            for (uint32_t k = 0; k < units(L); ++k, ++ub) {
                const int lk = L - 16 * (int)k;
                const W16 w = lds_w16(w32, src + 16 * (int)k, lk < 16 ? lk : 16);
                *reinterpret_cast<uint4 *>(dst + UNI_JP_OFF + 4 * ub) = make_uint4(w.x, w.y, w.z, w.w);
                auto conts = [](uint32_t x) { return __builtin_popcount(x & ~(x << 1) & 0x80808080u); };
                chars -= conts(w.x) + conts(w.y) + conts(w.z) + conts(w.w);
            }
            dst[UNI_JM_OFF + jb] = (uint32_t)L | (uint32_t)pos << 6 | base << 18;
            mywide += L > UNI_WMAX ? 1u : 0u;
            pos += L + chars + 1;
        }
    }
    {  // (and how many of them are wide: k_unigram_viterbi<true>'s)
        const uint32_t w = (uint32_t)lane_bcast((int)wave_incl_sum(mywide), 63);
        if (tid == 0) {
            dst[UNI_JN_OFF] = njobs;
            dst[UNI_JN_OFF + 1] = w;
        }
    }
#ifdef SDL_STAMPS
    if (tid == 0) {
        UNI_COUNT(0, 1);
        UNI_COUNT(1, np);
        UNI_COUNT(2, njobs);
        UNI_COUNT(6, s_scratch[3]);
    }
#endif
    __syncthreads();  // (the payloads are read before the list is packed over the window)
    base = base0;
    // the list is packed in LDS first (window and arena are dead now) and
    // written as whole 16-B lanes: scattered 4-B non-temporal stores cost ~3x
    // the list's bytes in HBM writes
    constexpr uint32_t PK_CAP = (uint32_t)(WIN_PAD + ARENA + 32) / 4 - 3;
    const bool packed = total <= PK_CAP;
    lds_u32 *pk = (lds_u32 *)s_bytes;
    for (int i = a0; i < a1; ++i) {
        const int prel = s_pieces[i] & 0xFFF;
        const uint32_t c = s_cnt[i];
        if (c == CNT_LONG) {
            const uint32_t it = atomicAdd(&counters[0], 1u);
            if (it < item_cap) items[it] = make_uint4((uint32_t)ci, base, (uint32_t)prel, s_stage[prel]);
            else atomicOr(err, 8u);
            if (packed) pk[base] = LMARK;
            else dst[base] = LMARK;
            ++base;
            continue;
        }
        const uint32_t k = ents(c);
        if (c & CNT_JOB) {  // placeholders: k_unigram_viterbi writes the entries
            for (uint32_t j = 0; j < k; ++j) {
                if (packed) pk[base + j] = LMARK | UNI_JOB_BIT;
                else dst[base + j] = LMARK | UNI_JOB_BIT;
            }
        } else if (packed) {
            for (uint32_t j = 0; j < k; ++j) pk[base + j] = (uint32_t)s_stage[prel + j];
        } else {
            for (uint32_t j = 0; j < k; ++j) __builtin_nontemporal_store((uint32_t)s_stage[prel + j], dst + base + j);
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
    uint16_t *const s_poff = s_stage;
    base = base0;
    for (int i = a0; i < a1; ++i) {
        s_poff[i] = (uint16_t)base;
        base += ents(s_cnt[i]);
    }
    __syncthreads();
    if (tid == 0) chunk_cnt[ci] = chunk_ent[ci] = total;
    // record boundaries owned by this chunk: entry offset of the first piece at
    // or after the boundary (k_unigram_long adds long items' extra ids)
    const int k_lo = (int)(r_lo - ra);
    for (int k = k_lo + tid; ra + k <= R; k += TOK_THREADS) {
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
    UNI_STAMP(5);
}

// ---------------------------------------------------------------------------
// k_unigram_viterbi: the Viterbi of every job the chunk kernel handed over -- word-table
// misses and medium words' pieces, "▁" + a payload of <= UNI_WMAX bytes -- one wave per
// chunk, the chunk's jobs in passes (its next jobs whose candidates fit VTCAP, <= VJP):
//   - candidate probes: every (start, end) candidate of every job of the pass is one task,
//     VU consecutive tasks a lane with all VU probes in flight; each task's exact f64 score
//     (-inf: no piece there) and id land in LDS at the task's index;
//   - DP, a lane per job, the nodes' f64 scores and back pointers in registers: the starts
//     ("▁", then payload bytes 0 .. 15) and their candidates' ends are compile-time loops,
//     so a node is a register and a candidate is one LDS load (its row's task base + end)
//     and a compare -- unigram_viterbi's visit order (starts, then ends ascending, then the
//     start's unk when no one-char piece starts there), strict-> and f64 sums;
//   - backtrack with unk fusion (a fused run is probed whole) from the back pointers in LDS;
//     the ids go to the chunk's results region at the job's stage position and its list
//     entry becomes LMARK | UNI_JOB_BIT | k << 24 | pos (k_compact_tokens expands it).
// Then the chunk's id count and its records' local offsets grow by the jobs' k - 1.
constexpr int UNI_VWAVES = 4;
// WIDE = false: the jobs of <= UNI_WMAX payload bytes (20 nodes, every one a register); true: the
// printable ASCII words of UNI_WMAX < L <= UNI_VMAX (nodes in a ring of UNI_VRING registers).  Two
// launches over the same job lists, so the common narrow jobs keep the small DP.
template <bool WIDE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(UNI_VWAVES, 8))) void k_unigram_viterbi(
    DevTok T, int64_t N, const uint64_t *__restrict__ off, int64_t R, const uint32_t *__restrict__ ranges,
    uint32_t *__restrict__ tokc, uint32_t *__restrict__ chunk_cnt, uint32_t *__restrict__ rec_local) {
    __shared__ __attribute__((aligned(16))) uint8_t s_pb[UNI_VPC * 16 + 32];  // payload units (+ lds_w16's reach)
    __shared__ uint32_t s_jm[VP_CAP];      // this launch's jobs: metas (L | pos << 6 | entry << 18)
    __shared__ uint16_t s_tb[VP_CAP + 1];  // task base of each job
    __shared__ uint8_t s_uo[VP_CAP];       // first payload unit of each job
    __shared__ uint8_t s_k[VP_CAP];        // ids of each job
    using CM = std::conditional_t<WIDE, uint64_t, uint32_t>;  // (<= UNI_VMAX / UNI_WMAX payload bytes)
    __shared__ CM s_cm[VP_CAP];            // bit x: payload byte x continues a char
    // wide passes (<= PFX_JOBS jobs): each payload start's prefix bound (T.upfx)
    __shared__ uint8_t s_pl[WIDE ? PFX_JOBS * UNI_VMAX : 1];
    __shared__ double s_sc[VTCAP];         // per task of the pass: the candidate's score, -inf: no piece
    __shared__ uint16_t s_id[VTCAP];       // ... its id
    // after the DP: back pointers (narrow: start node << 11 | task, UNK_T: unk, 0xFFFF: unset, per
    // node; wide: the words of 6-bit fields) [..][lane], over the dead scores
    constexpr int BPW = (UNI_VMAX + 4 + 4) / 5;
    uint16_t *const s_bp = reinterpret_cast<uint16_t *>(s_sc);
    uint32_t *const s_bpw = reinterpret_cast<uint32_t *>(s_sc);
    static_assert(UNI_NODES * 64 * 2 <= VTCAP * 8 && BPW * 64 * 4 <= VTCAP * 8, "the back pointers fit the scores' LDS");
    constexpr uint32_t UNK_T = 0x7FFu;
    constexpr int RG = UNI_VRING;
    static_assert(UNI_WMAX + 3 < UNI_NODES && UNI_NODES <= RG, "narrow jobs' nodes");
    const int lane = lane_id();
    const int64_t c = blockIdx.x;
    uint32_t *const slice = tokc + c * UNI_STAGE;
#ifdef SDL_STAMPS
    unsigned long long vstamp_ = __builtin_amdgcn_s_memtime();
#endif
    const uint32_t nall = slice[UNI_JN_OFF], nw = slice[UNI_JN_OFF + 1];
    if ((WIDE ? nw : nall - nw) == 0) return;
    const int Mm = T.maxlen_meta, Mf = T.maxlen_first;
    const int nj_all = (int)(nall < (uint32_t)VP_CAP ? nall : (uint32_t)VP_CAP);
    auto units = [](int L) -> uint32_t { return L > 16 ? (uint32_t)(L + 15) >> 4 : 1u; };
    // This launch's jobs, longest payload first: a pass's DP walks every start of its longest
    // job, so passes of like lengths (the short jobs together) cost less than list order's
    // mixed ones.  The order is free: each job's ids, entry and count fixups are its own.
    int njobs;
    static_assert(VP_CAP <= 128, "the chunk's jobs are two lane groups at most");
    {
        uint32_t ucarry = 0, jmv[2], uov[2], tv[2];
        int keyv[2];  // payload length of a job of this launch, -1 otherwise
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const int v = 64 * g + lane;
            const uint32_t jm = v < nj_all ? slice[UNI_JM_OFF + v] : 0u;
            const int L = (int)(jm & 63u);
            const bool mine = v < nj_all && (L > UNI_WMAX) == WIDE;
            const uint32_t un = v < nj_all ? units(L) : 0u;
            const uint32_t uincl = wave_incl_sum(un);
            jmv[g] = jm;
            uov[g] = ucarry + uincl - un;  // (payload units are laid out in list order)
            tv[g] = mine ? (uint32_t)vp_tasks(L, Mm, Mf) : 0u;
            keyv[g] = mine ? L : -1;
            ucarry += (uint32_t)lane_bcast((int)uincl, 63);
        }
        int x = 0;
        for (int k = WIDE ? UNI_VMAX : UNI_WMAX; k >= (WIDE ? UNI_WMAX + 1 : 0); --k) {
#pragma unroll
            for (int g = 0; g < 2; ++g) {
                const uint64_t m = __ballot(keyv[g] == k);
                if (keyv[g] == k) {
                    const int at = x + __popcll(m & ((1ull << lane) - 1ull));
                    s_jm[at] = jmv[g];
                    s_uo[at] = (uint8_t)uov[g];
                    s_tb[at] = (uint16_t)tv[g];
                }
                x += __popcll(m);
            }
        }
        njobs = x;
        __syncthreads();
        uint32_t carry = 0;  // task bases, in the sorted order
        for (int v0 = 0; v0 < njobs; v0 += 64) {
            const int v = v0 + lane;
            const uint32_t t = v < njobs ? (uint32_t)s_tb[v] : 0u, tincl = wave_incl_sum(t);
            if (v < njobs) s_tb[v] = (uint16_t)(carry + tincl - t);
            carry += (uint32_t)lane_bcast((int)tincl, 63);
        }
        if (lane == 0) s_tb[njobs] = (uint16_t)carry;
        const int nu = (int)(ucarry < (uint32_t)UNI_VPC ? ucarry : (uint32_t)UNI_VPC);
        for (int q = lane; q < nu; q += 64)
            *reinterpret_cast<uint4 *>(s_pb + 16 * q) = *reinterpret_cast<const uint4 *>(slice + UNI_JP_OFF + 4 * q);
        if (lane < 8) reinterpret_cast<uint32_t *>(s_pb + 16 * UNI_VPC)[lane] = 0u;
#ifdef SDL_STAMPS
        if (lane == 0) UNI_COUNT(3, carry);
#endif
    }
    __syncthreads();
    const lds_u8 *pb = (const lds_u8 *)s_pb;
    const lds_u32 *pb32 = (const lds_u32 *)s_pb;
    for (int v = lane; v < njobs; v += 64) {  // continuation bytes (10xxxxxx) of each payload
        const int L = (int)(s_jm[v] & 63u), u0 = s_uo[v];
        uint64_t m = 0;
        for (int k = 0; k < (L + 3) >> 2; ++k) {
            const uint32_t x = pb32[4 * u0 + k];
            m |= (uint64_t)gather4(x & ~(x << 1) & B7) << (4 * k);
        }
        s_cm[v] = (CM)(L < 64 ? m & ((1ull << L) - 1u) : m);
    }
    __syncthreads();
    VIT_STAMP(1);
    for (int a = 0; a < njobs;) {
        int b = a + 1;  // the pass: jobs [a, b)
        while (b < njobs && b - a < (WIDE ? PFX_JOBS : VJP) && (int)s_tb[b + 1] - (int)s_tb[a] <= VTCAP) ++b;
        const int T0 = s_tb[a], TZ = s_tb[b];
        if constexpr (WIDE) {  // the pass's starts' prefix bounds: one load each, all in flight
            for (int q = lane; q < (b - a) * UNI_VMAX; q += 64) {
                const int jl = q / UNI_VMAX, i = q - jl * UNI_VMAX;
                const int Lq = (int)(s_jm[a + jl] & 63u);
                uint32_t bound = 255u;  // (fewer than 4 bytes left: no candidate to bound)
                if (i + 4 <= Lq) bound = T.upfx[uni_pfx_key(lds_w16(pb32, 16 * s_uo[a + jl] + i, 4).x)];
                s_pl[q] = (uint8_t)bound;
            }
            __syncthreads();
        }
        {  // lane l takes the pass's tasks [T0 + l K, T0 + (l + 1) K) in rounds of VU: one
           // decode per pass, then (i, j) steps along the rows; a row's 16 bytes are read once
        const int K = (TZ - T0 + 63) >> 6;
        const int tl0 = T0 + lane * K, tl1 = tl0 + K < TZ ? tl0 + K : TZ;
        int jv = a, i = -1, j = -1, L = 0, src = 0;
        CM cm = 0;  // the job's continuation-byte mask
        if (tl0 < tl1) {
            int lo = a, hi = b - 1;  // the job holding task tl0
            while (lo < hi) {
                const int m = (lo + hi + 1) >> 1;
                if ((int)s_tb[m] <= tl0) lo = m; else hi = m - 1;
            }
            jv = lo;
            L = (int)(s_jm[jv] & 63u);
            src = 16 * s_uo[jv];
            cm = s_cm[jv];
            vp_decode(tl0 - (int)s_tb[jv], L, Mm, Mf, &i, &j);
            --j;  // (the first step lands on it)
        }
        int cur_ps = -1;
        W16 rowb{0, 0, 0, 0};
        for (int r0 = tl0; r0 < tl0 + K; r0 += VU) {  // (K is wave-uniform)
            Probe P[VU];
            W16 W[VU];
            uint32_t meta[VU];  // n | cont << 8 | (n > 16: payload byte of its start) << 12; ~0u: no probe
#pragma unroll
            for (int u = 0; u < VU; ++u) {
                meta[u] = ~0u;
                W[u] = W16{0, 0, 0, 0};
                if (r0 + u >= tl1) continue;
                // the next candidate: (i, j + 1), else the next row / job
                ++j;
                const int jmax = i < 0 ? (L < Mm ? L : Mm) : (L < i + Mf ? L : i + Mf);
                if (j > jmax) {
                    ++i;
                    j = i + 1;
                    if (i >= L) {
                        ++jv;
                        L = (int)(s_jm[jv] & 63u);
                        src = 16 * s_uo[jv];
                        cm = s_cm[jv];
                        i = -1;
                        j = 0;
                    }
                }
                // candidates start and end on char boundaries
                if (((i > 0 ? cm >> i : (CM)0) | cm >> j) & 1u) continue;
                const int ps = i < 0 ? 0 : i;
                const int n = j - ps;
                // (wide rows: no plain piece this long starts with these 4 bytes)
                if constexpr (WIDE)
                    if (i >= 0 && n >= 4 && n > (int)s_pl[(jv - a) * UNI_VMAX + i]) continue;
                const uint32_t cont = i < 0 ? UC_META : UC_PIECE;
                meta[u] = (uint32_t)n | cont << 8;
                if (src + ps != cur_ps) {
                    cur_ps = src + ps;
                    rowb = lds_w16(pb32, cur_ps, 16);
                }
                W[u] = keep_bytes(rowb, n);
                if (!WIDE || n <= 16) {
                    P[u] = probe_load(T, hash16(W[u], (uint32_t)n, cont));
                } else {  // (rows of wide jobs: pieces of 17 .. maxlen_first bytes) two blocks; the
                          // bytes past 16 are checked against the vocab pool on a header match
                    const W16 w2 = lds_w16(pb32, cur_ps + 16, n - 16);
                    uint32_t h = hinit((uint32_t)n, cont);
                    h = hmix(hmix(hmix(hmix(h, W[u].x), W[u].y), W[u].z), W[u].w);
                    h = hmix(hmix(hmix(hmix(h, w2.x), w2.y), w2.z), w2.w);
                    P[u] = probe_load(T, hfinal(h));
                    meta[u] |= (uint32_t)cur_ps << 12;
                }
            }
#pragma unroll
            for (int u = 0; u < VU; ++u) {
                const int t = r0 + u;
                if (t >= tl1) continue;
                double sc = -__builtin_inf();
                if (meta[u] != ~0u) {
                    uint32_t w3 = 0;
                    int id = probe_result_w3(P[u], meta[u] & 0x3FFu, W[u], &w3);
                    if constexpr (WIDE) {
                        const uint32_t n = meta[u] & 31u;
                        if (n > 16 && id >= 0) {  // (the slot matched length, cont and the first 16 bytes)
                            const int q0 = (int)(meta[u] >> 12);
                            const uint32_t key = meta[u] & 0x3FFu;
                            const bool m1 = slot_match(P[u].a1, P[u].b1, key, W[u]);
                            const uint32_t z = m1 ? P[u].a1.z : P[u].a2.z;
                            for (uint32_t x = 16; x < n && id >= 0; ++x)
                                if (T.vpool[z + x] != pb[q0 + (int)x]) id = -1;
                            if (id < 0 && m1 && slot_match(P[u].a2, P[u].b2, key, W[u])) {  // (both: the second)
                                id = (int32_t)P[u].a2.y;
                                w3 = P[u].a2.w;
                                for (uint32_t x = 16; x < n && id >= 0; ++x)
                                    if (T.vpool[P[u].a2.z + x] != pb[q0 + (int)x]) id = -1;
                            }
                        }
                    }
                    if (id >= 0) {
                        sc = uni_score64(__uint_as_float(w3), (uint32_t)id);
                        s_id[t - T0] = (uint16_t)((uint32_t)id & UNI_ID_MASK);
                    }
                }
                s_sc[t - T0] = sc;
            }
        }
        }
        __syncthreads();
        VIT_STAMP(2);
        // -- DP: a lane per job --
        const bool act = lane < b - a;
        const int v = act ? a + lane : a;
        const uint32_t jm = act ? s_jm[v] : 0u;
        const int L = (int)(jm & 63u), n = L + 3;
        int Lmax = L;  // the pass's longest payload (wave-uniform bound of the loops)
#pragma unroll
        for (int k = 1; k < 64; k <<= 1) {
            const int o = __shfl_xor(Lmax, k);
            Lmax = o > Lmax ? o : Lmax;
        }
        const int src = 16 * s_uo[v];
        const int tj = (int)s_tb[v] - T0;  // the job's first task in the pass
        const int c0 = vp_c0(L, Mm);
        const uint32_t pos = (jm >> 6) & 0xFFFu;
        uint16_t *const jr = reinterpret_cast<uint16_t *>(slice + UNI_JR_OFF) + pos;
        auto acc = [&](int x) -> uint32_t { return x < 3 ? meta_byte(x) : (uint32_t)pb[src + x - 3]; };
        auto cand = [&](int st2, int e2, double *) -> int {  // the fused-unk lookup
            int id;
            if (st2 == 0) id = e2 - 3 <= Mm ? probe_acc(T, acc, 3, e2 - 3, UC_META) : -1;
            else id = e2 - st2 <= Mf ? probe_acc(T, acc, st2, e2 - st2, UC_PIECE) : -1;
            return uni_piece_id(id);
        };
        int k = 0;
        if constexpr (!WIDE) {
            // The nodes' f64 scores and back pointers in registers: the starts ("▁", then payload
            // bytes 0 .. 15) and their candidates' ends are compile-time loops, so a node is a
            // register and a candidate is one LDS load (its row's task base + end) and a compare
            // -- unigram_viterbi's visit order (starts, then ends ascending, then the start's unk
            // when no one-char piece starts there), strict-> and f64 sums.
            const uint4 pw = *reinterpret_cast<const uint4 *>(s_pb + src);
            double best[UNI_NODES];
            uint32_t bp[UNI_NODES];
            static_for<0, UNI_NODES>([&](auto X) {
                best[X] = -__builtin_inf();
                bp[X] = 0xFFFFu;
            });
            auto relax = [&](auto E, double cc, uint32_t bb) {
                const bool up = cc > best[E];
                best[E] = up ? cc : best[E];
                bp[E] = up ? bb : bp[E];
            };
            {  // start 0: "▁" + payload[0, j), j = 0 .. min(L, Mm) = tasks tj + j, ending at node 3 + j
                const int jz = L < Mm ? L : Mm;
                static_for<0, UNI_WMAX + 1>([&](auto J) {
                    constexpr int jj = decltype(J)::value;
                    if (jj <= Lmax && act && jj <= jz) relax(std::integral_constant<int, 3 + jj>{}, s_sc[tj + jj],
                                                              (uint32_t)(tj + jj));
                });
                // the "▁" char's unk when "▁" is no piece
                if (act && !(s_sc[tj] > -__builtin_inf())) relax(std::integral_constant<int, 3>{}, T.unk_score, UNK_T);
            }
            static_for<0, UNI_WMAX>([&](auto I) {  // payload start i = node 3 + i
                constexpr int i = decltype(I)::value, st = 3 + i;
                if (i < Lmax) {
                    const uint32_t by = ((i < 4 ? pw.x : i < 8 ? pw.y : i < 12 ? pw.z : pw.w) >> (8 * (i & 3))) & 0xFFu;
                    const bool on = act && i < L && (i == 0 || (by & 0xC0u) != 0x80u);
                    const double base = best[st];
                    const int rlen = L - i < Mf ? L - i : Mf;
                    const int rb = tj + c0 + vp_rowoff(i, L, Mf);
                    static_for<1, UNI_WMAX - i + 1>([&](auto D) {
                        constexpr int d = decltype(D)::value;
                        if (on && d <= rlen)
                            relax(std::integral_constant<int, st + d>{}, s_sc[rb + d - 1] + base,
                                  (uint32_t)st << 11 | (uint32_t)(rb + d - 1));
                    });
                    const int l0 = u8len_lead(by), mb = l0 < L - i ? l0 : L - i;
                    if (on && !(mb <= rlen && s_sc[rb + mb - 1] > -__builtin_inf())) {  // unk: no one-char piece
                        static_for<1, 5>([&](auto M) {
                            constexpr int m = decltype(M)::value;
                            if constexpr (st + m < UNI_NODES)
                                if (mb == m) relax(std::integral_constant<int, st + m>{}, T.unk_score + base,
                                                   (uint32_t)st << 11 | UNK_T);
                        });
                    }
                }
            });
            // -- backtrack (the back pointers to LDS: the scores are dead) --
            static_for<0, UNI_NODES>([&](auto X) { s_bp[X * 64 + lane] = (uint16_t)bp[X]; });
            VIT_STAMP(3);
            if (act) {
                struct {
                    const uint16_t *bp;
                    const uint16_t *id16;
                    int lane, unk;
                    __device__ int start(int x) const {
                        const uint32_t b = bp[x * 64 + lane];
                        return b == 0xFFFFu ? -1 : (int)(b >> 11);
                    }
                    __device__ int id(int x) const {
                        const uint32_t b = bp[x * 64 + lane];
                        return b == 0xFFFFu ? -1 : (b & 0x7FFu) == UNK_T ? unk : (int)id16[b & 0x7FFu];
                    }
                } nodes{s_bp, s_id, lane, T.unk_id};
                k = unigram_backtrack(n, cand, nodes, T.unk_id, [&](int x, int id) { jr[x] = (uint16_t)id; });
            }
        } else {
            // Few jobs a pass (~3 a held-out chunk), each up to UNI_VMAX + 3 nodes: a group of 21
            // lanes per job, 3 jobs at a time.  The starts are visited in order; lane d of the
            // group relaxes the start's candidate ending d + 1 bytes on (distinct nodes), its last
            // lane the start's unk (when no one-char piece starts there, so never a node a piece
            // of the same start reaches) -- unigram_viterbi's relaxations, strict-> and f64 sums,
            // the nodes (f64 score, start << 16 | task) in LDS; lane 0 of the group backtracks.
            constexpr int GN = UNI_VMAX + 4, GL = 21;
            __shared__ double s_gb[3 * GN];
            __shared__ uint32_t s_gp[3 * GN];
            auto wave_sync = [] {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            };
            const int grp = lane / GL, gl = lane - GL * grp;  // (lane 63: no group)
            for (int j0 = a; j0 < b; j0 += 3) {
                const int vj = j0 + grp;
                const bool gact = grp < 3 && vj < b;
                const uint32_t jmg = gact ? s_jm[vj] : 0u;
                const int Lg = (int)(jmg & 63u), ng = gact ? Lg + 3 : 0;
                const int srcg = gact ? 16 * s_uo[vj] : 0, tjg = gact ? (int)s_tb[vj] - T0 : 0;
                const int c0g = vp_c0(Lg, Mm);
                const uint64_t cmg = gact ? s_cm[vj] : 0ull;
                lds_f64 *gb = (lds_f64 *)s_gb + (grp < 3 ? grp : 0) * GN;
                lds_u32 *gp = (lds_u32 *)s_gp + (grp < 3 ? grp : 0) * GN;
                for (int x = gl; gact && x <= ng; x += GL) {
                    gb[x] = x == 0 ? 0.0 : -__builtin_inf();
                    gp[x] = 0xFFFFFFFFu;
                }
                int nmax = ng;  // (wave-uniform bound of the start loop)
#pragma unroll
                for (int q = 1; q < 64; q <<= 1) {
                    const int o = __shfl_xor(nmax, q);
                    nmax = o > nmax ? o : nmax;
                }
                wave_sync();
                auto relaxg = [&](int e, double cc, uint32_t bb) {
                    if (gp[e] == 0xFFFFFFFFu || cc > gb[e]) {
                        gb[e] = cc;
                        gp[e] = bb;
                    }
                };
                for (int st = 0; st < nmax; st = st == 0 ? 3 : st + 1) {
                    const int i = st - 3;
                    if (gact && st < ng && (st == 0 || !((cmg >> i) & 1u))) {
                        const double base = gb[st];
                        const int rlen = st == 0 ? (Lg < Mm ? Lg : Mm) + 1 : (Lg - i < Mf ? Lg - i : Mf);
                        const int rb = st == 0 ? tjg : tjg + c0g + vp_rowoff(i, Lg, Mf);
                        if (gl < rlen && gl < GL - 1) {  // candidate (st, e): "▁" row ends 3 + gl, else st + gl + 1
                            const int t = rb + gl, e = st == 0 ? 3 + gl : st + gl + 1;
                            const double sv = s_sc[t];
                            if (sv > -__builtin_inf()) relaxg(e, sv + base, (uint32_t)st << 16 | (uint32_t)t);
                        }
                        if (gl == GL - 1) {  // unk
                            const int l0 = st == 0 ? 3 : u8len_lead(pb[srcg + i]), mb = l0 < ng - st ? l0 : ng - st;
                            const int ts = st == 0 ? rb : rb + mb - 1;  // the one-char piece's task
                            if (!((st == 0 || mb <= rlen) && s_sc[ts] > -__builtin_inf()))
                                relaxg(st + mb, T.unk_score + base, (uint32_t)st << 16 | UNK_T);
                        }
                    }
                    wave_sync();
                }
                if (gact && gl == 0) {
                    struct {
                        const uint32_t *gp;
                        const uint16_t *id16;
                        int unk;
                        __device__ int start(int x) const { return gp[x] == 0xFFFFFFFFu ? -1 : (int)(gp[x] >> 16); }
                        __device__ int id(int x) const {
                            const uint32_t b = gp[x];
                            return b == 0xFFFFFFFFu ? -1 : (b & 0xFFFFu) == UNK_T ? unk : (int)id16[b & 0xFFFFu];
                        }
                    } nodes{(const uint32_t *)gp, s_id, T.unk_id};
                    auto accg = [&](int x) -> uint32_t { return x < 3 ? meta_byte(x) : (uint32_t)pb[srcg + x - 3]; };
                    auto candg = [&](int st2, int e2, double *) -> int {
                        int id;
                        if (st2 == 0) id = e2 - 3 <= Mm ? probe_acc(T, accg, 3, e2 - 3, UC_META) : -1;
                        else id = e2 - st2 <= Mf ? probe_acc(T, accg, st2, e2 - st2, UC_PIECE) : -1;
                        return uni_piece_id(id);
                    };
                    const uint32_t posg = (jmg >> 6) & 0xFFFu;
                    uint16_t *const jrg = reinterpret_cast<uint16_t *>(slice + UNI_JR_OFF) + posg;
                    const int kg = unigram_backtrack(ng, candg, nodes, T.unk_id, [&](int x, int id) { jrg[x] = (uint16_t)id; });
                    slice[jmg >> 18] = LMARK | UNI_JOB_BIT | (uint32_t)kg << 24 | posg;
                    s_k[vj] = (uint8_t)kg;
                }
                wave_sync();
            }
            VIT_STAMP(3);
        }
        if (!WIDE && act) {
            slice[jm >> 18] = LMARK | UNI_JOB_BIT | (uint32_t)k << 24 | pos;
            s_k[v] = (uint8_t)k;
        }
#ifdef SDL_STAMPS
        if (lane == 0) UNI_COUNT(4, 1);
#endif
        __syncthreads();
        VIT_STAMP(4);
        a = b;
    }
    // the chunk's id count and its records' local offsets: + (k - 1) of every job before them
    uint32_t ext = 0;
    for (int v = lane; v < njobs; v += 64) ext += (uint32_t)s_k[v] - 1u;
    ext = (uint32_t)lane_bcast((int)wave_incl_sum(ext), 63);
    if (lane == 0 && ext) atomicAdd(&chunk_cnt[c], ext);
    const int64_t c0 = c * CHUNK, c1 = c0 + CHUNK < N ? c0 + CHUNK : N;
    for (int64_t r = ranges[3 * c + 2]; r <= R; ++r) {
        const int64_t p = (int64_t)off[r];
        if (p >= c1) break;
        uint32_t add = 0;
        for (int v = lane; v < njobs; v += 64)
            if ((int64_t)((s_jm[v] >> 6) & 0xFFFu) < p - c0) add += (uint32_t)s_k[v] - 1u;
        add = (uint32_t)lane_bcast((int)wave_incl_sum(add), 63);
        if (lane == 0 && add) atomicAdd(&rec_local[r], add);
    }
    VIT_STAMP(5);
}

namespace {
constexpr size_t huge_scratch_bytes() {
    return (size_t)UNI_HUGE_NORM + sizeof(UniNode) * (UNI_HUGE_NORM + 8) + 4 * (2 * UNI_HUGE_NORM + 8);
}
__device__ Scratch make_scratch(uint8_t *mine, int cap) {
    return Scratch{mine + sizeof(UniNode) * (cap + 8) + 4 * (2 * cap + 8), reinterpret_cast<UniNode *>(mine),
                   reinterpret_cast<uint32_t *>(mine + sizeof(UniNode) * (cap + 8)), cap};
}
}  // namespace

// Long items, one wave each: the lanes stage the item's raw bytes (LONG_RAW
// from just before it) in LDS, lane 0 normalizes the word from there into LDS
// and walks its pieces; per piece, lanes take candidate rows (a start position
// each, up to Mf probes, 4 in flight) and lane 0 relaxes the nodes of those 64
// starts from LDS, then backtracks.  Items past LONG_NORM normalized bytes go
// to the huge list.  KMAX bounds a row's candidate ends (max(Mm + 1, Mf));
// the LDS footprint (~20 KB at KMAX 32) sets how many items a CU keeps in flight.
constexpr int LONG_NORM = 512;  // stage 2; stage 1 takes items of <= LONG_NORM1 normalized bytes
constexpr int LONG_NORM1 = 128;
constexpr int LONG_UNROLL = 2;  // candidate probes in flight per lane (k_unigram_long)
constexpr int LONG_RAW = 1024;

template <int KMAX, int NORM>
__global__ __launch_bounds__(64) void k_unigram_long(DevTok T, const uint8_t *__restrict__ text, int64_t N,
                                                     const uint64_t *__restrict__ off, int64_t R,
                                                     const uint32_t *__restrict__ ranges,
                                                     const uint4 *__restrict__ items, uint32_t item_cap,
                                                     const uint32_t *n_in, uint32_t *counters, uint32_t *tokc,
                                                     uint32_t *chunk_cnt, uint32_t *rec_local, uint32_t *pool,
                                                     uint32_t pool_cap, uint4 *over, uint32_t over_cap,
                                                     uint32_t *n_over, uint32_t *err) {
    __shared__ __attribute__((aligned(16))) uint8_t s_nb[NORM + 32];
    __shared__ double s_sc[NORM + 8];
    __shared__ uint32_t s_st[NORM + 8];  // node start | id << 16 (0xFFFF: unset)
    __shared__ uint16_t s_ids[2 * NORM + 16];
    __shared__ uint16_t s_cid[KMAX * 64];     // [k][lane]: id of row lane's k-th end
    __shared__ __attribute__((aligned(16))) float s_csc[KMAX * 64];
    // the item's raw bytes are staged where the candidate scores go later (the
    // normalization is done before the first probe): 1 KB less LDS per item
    static_assert(KMAX * 64 * 4 >= LONG_RAW, "raw staging aliases s_csc");
    uint8_t *const s_raw = reinterpret_cast<uint8_t *>(s_csc);
    __shared__ unsigned long long s_mask[64];
    __shared__ int s_misc[8];
    const int lane = lane_id();
    lds_u8 *nb = (lds_u8 *)s_nb;
    const lds_u32 *w32 = (const lds_u32 *)s_nb;
    const int Mm = T.maxlen_meta, Mf = T.maxlen_first;
    uint32_t n_items = *n_in;
    if (n_items > item_cap) n_items = item_cap;
#ifdef SDL_STAMPS
    unsigned long long lstamp_ = __builtin_amdgcn_s_memtime();
#endif
    for (uint32_t it_i = blockIdx.x; it_i < n_items; it_i += gridDim.x) {
        const uint4 it = items[it_i];
        const int64_t p = (int64_t)it.x * CHUNK + it.z;
        // the record holding p: between the last one starting before its chunk
        // and the first one starting past its window (k_chunk_ranges)
        const int64_t r_lo = ranges[3 * (int64_t)it.x + 2], r_hi = ranges[3 * (int64_t)it.x + 1];
        const int64_t rec = record_of(off, R, p, r_lo > 0 ? r_lo - 1 : 0, (r_hi < R ? r_hi : R) - 1);
        const int64_t pa = (p - 1) & ~(int64_t)15;  // staged raw bytes: [pa, pa + LONG_RAW)
        *reinterpret_cast<uint4 *>(s_raw + 16 * lane) = load16(text, pa + 16 * lane, N);
        __syncthreads();
        const int64_t rs = (int64_t)off[rec];
        const int64_t re = (int64_t)off[rec + 1] < N ? (int64_t)off[rec + 1] : N;
        const lds_u8 *raw = (const lds_u8 *)s_raw;
        auto byte = [&](int64_t q) -> uint32_t {
            return (uint64_t)(q - pa) < (uint64_t)LONG_RAW ? (uint32_t)raw[q - pa] : (uint32_t)text[q];
        };
        // the raw word's end (word_end_b), the wave scanning 64 bytes a step
        int64_t end = it.w ? p + it.w : -1;
        for (int64_t q0 = p + 1; end < 0; q0 += 64) {
            const int64_t q = q0 + lane;
            bool stop = q >= re;
            if (!stop) {
                const uint32_t b = byte(q);
                int l;
                auto bnd = [&](int64_t x) -> bool { return x >= re; };
                stop = ascii_ws(b) || (b == (uint32_t)'<' && T.n_special && uni_special(T, q, N, byte, bnd, &l) >= 0);
            }
            const uint64_t m = __ballot(stop);
            if (m) end = q0 + __builtin_ctzll(m);
        }
        // a word of printable ASCII is its own normalization (host-checked
        // charsmap facts, as the chunk kernel's simple words): copied by the wave
        const int wl = (int)(end - p);
        bool ascii = wl <= NORM && p - pa + wl <= LONG_RAW;
        if (ascii) {
            bool mine = true;
            for (int j = lane; j < wl; j += 64) mine = mine && (uint32_t)s_raw[p - pa + j] - 0x21u < 0x5Eu;
            ascii = !__any(!mine);
        }
        if (ascii) {
            for (int j = lane; j < wl + 8; j += 64) nb[j] = j < wl ? s_raw[p - pa + j] : (uint8_t)0;
            if (lane == 0) {
                s_misc[0] = wl;
                s_misc[1] = 0;
                s_misc[5] = 0;
                s_misc[6] = -1;
                s_misc[7] = 0;
            }
        } else if (lane == 0) {
            int nl = 0;
            const bool ok = normalize_span(T, byte, p, end, p > rs && byte(p - 1) == (uint32_t)' ',
                                           [&](uint32_t x) -> bool {
                                               if (nl >= NORM) return false;
                                               nb[nl++] = (uint8_t)x;
                                               return true;
                                           });
            for (int z = 0; z < 8; ++z) nb[nl + z] = 0;
            s_misc[0] = ok ? nl : -1;
            s_misc[1] = 0;  // cursor: where the next word/piece search starts
            s_misc[5] = 0;  // ids so far
            s_misc[6] = -1; // end of the current word (-1: none)
            s_misc[7] = 0;  // the current piece is virtual-"▁"-prefixed
        }
        __syncthreads();
        const int nl = s_misc[0];
        LONG_COUNT(0, 1);
        LONG_COUNT(1, ascii ? 1 : 0);
        LONG_STAMP(1);
        if (nl < 0) {
            if (lane == 0) {
                const uint32_t h = atomicAdd(n_over, 1u);  // normalized past NORM: the next stage
                if (h < over_cap) over[h] = it;
                else atomicOr(err, 8u);
            }
            __syncthreads();
            continue;
        }
        auto nbr = [&](int i) -> uint32_t { return nb[i]; };
        for (;;) {
            // lane 0: the next Metaspace piece -> (payload src, length) or done
            if (lane == 0) {
                int cur = s_misc[1], wend = s_misc[6];
                int src = -1, L = 0;
                if (wend < 0 || cur >= wend) {  // next word
                    int l;
                    while (cur < nl && norm_ws(T, nbr, cur, &l)) cur += l;
                    if (cur < nl) {
                        int j = cur;
                        while (j < nl && !norm_ws(T, nbr, j, &l)) j += l;
                        wend = j;
                        const bool m = j - cur >= 3 && nb[cur] == 0xE2 && nb[cur + 1] == 0x96 && nb[cur + 2] == 0x81;
                        s_misc[7] = m ? 0 : 1;
                    } else {
                        wend = -1;
                    }
                }
                if (wend >= 0) {
                    const bool virt = s_misc[7] != 0;
                    src = virt ? cur : cur + 3;  // payload after the "▁"
                    int t = cur + (virt ? 1 : 3);
                    while (t < wend && !(t + 3 <= wend && nb[t] == 0xE2 && nb[t + 1] == 0x96 && nb[t + 2] == 0x81)) ++t;
                    L = t - src;
                    cur = t;
                    s_misc[7] = 0;
                }
                s_misc[1] = cur;
                s_misc[6] = wend;
                s_misc[2] = src;
                s_misc[3] = L;
            }
            __syncthreads();
            const int src = s_misc[2], L = s_misc[3];
            LONG_STAMP(2);
            if (src < 0) break;
            LONG_COUNT(2, 1);
            LONG_COUNT(3, L);
            const int n = L + 3;  // the piece "▁" + payload
            for (int i = lane; i <= n; i += 64) {
                s_sc[i] = 0.0;
                s_st[i] = 0xFFFFFFFFu;
            }
            // acc / cand over the piece (cand: the fused-unk lookup, lane 0)
            auto acc = [&](int x) -> uint32_t { return x < 3 ? meta_byte(x) : (uint32_t)nb[src + x - 3]; };
            auto cand = [&](int st2, int e2, double *sc) -> int {
                int id;
                if (st2 == 0) id = (e2 - 3 <= Mm) ? probe_acc(T, nbr, src, e2 - 3, UC_META) : -1;
                else id = (e2 - st2 <= Mf) ? probe_acc(T, nbr, src + st2 - 3, e2 - st2, UC_PIECE) : -1;
                id = uni_piece_id(id);
                if (id >= 0) *sc = T.uscore[id];
                return id;
            };
            __syncthreads();
            for (int r0 = 0; r0 <= L; r0 += 64) {
                // the candidates of rows r0 .. r0 + 63 (row r: payload start r - 1, r == 0
                // the "▁" row) dealt to all lanes, 4 probes in flight each
                const int nrow = L + 1 - r0 < 64 ? L + 1 - r0 : 64;
                const int ta = r0 == 0 ? 0 : vp_c0(L, Mm) + vp_rowoff(r0 - 1, L, Mf);
                const int tz = r0 + nrow > L ? vp_tasks(L, Mm, Mf) : vp_c0(L, Mm) + vp_rowoff(r0 + nrow - 1, L, Mf);
                s_mask[lane] = 0ull;
                __syncthreads();
                for (int tq = ta; tq < tz; tq += 64 * LONG_UNROLL) {
                    Probe P[LONG_UNROLL];
                    W16 Wd[LONG_UNROLL];
                    int gen[LONG_UNROLL];
                    uint32_t gw3[LONG_UNROLL], meta[LONG_UNROLL];  // row | k << 8 | len << 16 | cont << 24; ~0u: none
#pragma unroll
                    for (int u = 0; u < LONG_UNROLL; ++u) {
                        const int t = tq + 64 * u + lane;
                        meta[u] = ~0u;
                        gen[u] = -2;
                        gw3[u] = 0;
                        Wd[u] = W16{0, 0, 0, 0};
                        if (t >= tz) continue;
                        int i, j;
                        vp_decode(t, L, Mm, Mf, &i, &j);
                        if ((i > 0 && (nb[src + i] & 0xC0u) == 0x80u) || (j < L && (nb[src + j] & 0xC0u) == 0x80u))
                            continue;  // candidates start and end on char boundaries
                        const int ps = i < 0 ? 0 : i;
                        const int len = j - ps;
                        const uint32_t cont = i < 0 ? UC_META : UC_PIECE;
                        meta[u] = (uint32_t)(i + 1 - r0) | (uint32_t)(i < 0 ? j : j - i - 1) << 8 | (uint32_t)len << 16 |
                                  cont << 24;
                        Wd[u] = lds_w16(w32, src + ps, len);
                        if (len <= 16) {
                            P[u] = probe_load(T, hash16(Wd[u], (uint32_t)len, cont));
                        } else if (len <= 32) {  // two blocks; bytes past 16 checked on a header match
                            const W16 w2 = lds_w16(w32, src + ps + 16, len - 16);
                            uint32_t h = hinit((uint32_t)len, cont);
                            h = hmix(hmix(hmix(hmix(h, Wd[u].x), Wd[u].y), Wd[u].z), Wd[u].w);
                            h = hmix(hmix(hmix(hmix(h, w2.x), w2.y), w2.z), w2.w);
                            P[u] = probe_load(T, hfinal(h));
                            gen[u] = -3;
                        } else {
                            gen[u] = probe_acc(T, nbr, src + ps, len, cont, &gw3[u]);
                        }
                    }
#pragma unroll
                    for (int u = 0; u < LONG_UNROLL; ++u) {
                        if (meta[u] == ~0u) continue;
                        uint32_t w3 = gw3[u];
                        const uint32_t key = ((meta[u] >> 16) & 0xFFu) | ((meta[u] >> 24) << 8);
                        int id;
                        if (gen[u] == -3) {  // 17..32 bytes: header + first 16 bytes, then the pool
                            id = -1;
                            const int len = (int)((meta[u] >> 16) & 0xFFu);
                            const int ps = (int)(meta[u] & 0xFFu) + r0 - 1;
                            for (int which = 0; which < 2 && id < 0; ++which) {
                                const uint4 sa = which ? P[u].a2 : P[u].a1, sb = which ? P[u].b2 : P[u].b1;
                                if (!slot_match(sa, sb, key, Wd[u])) continue;
                                bool ok = true;
                                for (int x = 16; x < len && ok; ++x) ok = T.vpool[sa.z + x] == nb[src + (ps < 0 ? 0 : ps) + x];
                                if (ok) {
                                    id = (int32_t)sa.y;
                                    w3 = sa.w;
                                }
                            }
                        } else {
                            id = gen[u] != -2 ? gen[u] : probe_result_w3(P[u], key, Wd[u], &w3);
                        }
                        if (id < 0) continue;
                        const int q = (int)(meta[u] & 0xFFu), k = (int)((meta[u] >> 8) & 0xFFu);
                        s_cid[k * 64 + q] = (uint16_t)id;
                        s_csc[k * 64 + q] = __uint_as_float(w3);  // the slot's f32 score (uni_score64; k < KMAX host-checked)
                        atomicOr(&s_mask[q], 1ull << k);
                    }
                }
                __syncthreads();
                LONG_STAMP(3);
                // relax the nodes from these rows' starts, in order; a row's candidates
                // end at distinct nodes, so lane k relaxes the row's k-th end
                const int rz = L + 1 - r0 < 64 ? L + 1 - r0 : 64;
                for (int q = 0; q < rz; ++q) {
                    const int r = r0 + q;
                    const int st = r == 0 ? 0 : r + 2;  // node position of the row's start
                    if (r > 1 && (nb[src + r - 1] & 0xC0u) == 0x80u) continue;
                    const int l0 = u8len_lead(acc(st));
                    const int mb = l0 < n - st ? l0 : n - st;
                    const double base = s_sc[st];
                    const int fe = st == 0 ? 3 : st + 1;
                    const unsigned long long m = s_mask[q];
                    const bool single = (m >> (st + mb - fe)) & 1ull;
                    if (lane < KMAX && ((m >> lane) & 1ull)) {
                        const int e = fe + lane;
                        const uint32_t id16 = s_cid[lane * 64 + q];
                        const double c = uni_score64(s_csc[lane * 64 + q], id16) + base;
                        if (s_st[e] == 0xFFFFFFFFu || c > s_sc[e]) {
                            s_sc[e] = c;
                            s_st[e] = (uint32_t)st | ((id16 & UNI_ID_MASK) << 16);
                        }
                    }
                    if (!single && lane == 63) {  // the unk candidate ends where no piece candidate does
                        const double c = T.unk_score + base;
                        const int e = st + mb;
                        if (s_st[e] == 0xFFFFFFFFu || c > s_sc[e]) {
                            s_sc[e] = c;
                            s_st[e] = (uint32_t)st | ((uint32_t)T.unk_id << 16);
                        }
                    }
                    __syncthreads();
                }
                __syncthreads();
                LONG_STAMP(4);
            }
            if (lane == 0) {
                struct {
                    const uint32_t *st;
                    __device__ int start(int i) const { return st[i] == 0xFFFFFFFFu ? -1 : (int)(st[i] & 0xFFFFu); }
                    __device__ int id(int i) const { return st[i] == 0xFFFFFFFFu ? -1 : (int)(st[i] >> 16); }
                } nodes{s_st};
                const int k0 = s_misc[5];
                const int k = unigram_backtrack(n, cand, nodes, T.unk_id, [&](int x, int id) {
                    if (k0 + x < 2 * NORM + 16) s_ids[k0 + x] = (uint16_t)id;
                });
                s_misc[5] = k0 + k;
            }
            __syncthreads();
            LONG_STAMP(5);
        }
        if (lane == 0) {
            int k = s_misc[5];
            if (k > 2 * NORM + 16) {
                atomicOr(err, 2u);
                k = 0;
            }
            finalize_item(it.x, it.y, p, rec, k, [&](int j) { return (uint32_t)s_ids[j]; }, off, R, tokc, chunk_cnt,
                          rec_local, pool, counters + 2, pool_cap, err);
        }
        __syncthreads();
        LONG_STAMP(6);
    }
}

// Items whose normalized text exceeds a lane's scratch: one wave each, lane 0.
__global__ __launch_bounds__(64) void k_unigram_huge(DevTok T, const uint8_t *__restrict__ text, int64_t N,
                                                     const uint64_t *__restrict__ off, int64_t R, uint32_t *counters,
                                                     uint32_t *tokc, uint32_t *chunk_cnt, uint32_t *rec_local,
                                                     uint8_t *scratch, uint32_t *pool, uint32_t pool_cap,
                                                     const uint4 *huge, uint32_t huge_cap, uint32_t *err) {
    if (lane_id() != 0) return;
    const Scratch S = make_scratch(scratch + (size_t)blockIdx.x * huge_scratch_bytes(), UNI_HUGE_NORM);
    uint32_t nh = counters[3];
    if (nh > huge_cap) nh = huge_cap;
    for (uint32_t i = blockIdx.x; i < nh; i += gridDim.x) {
        const uint4 h = huge[i];
        const int64_t p = (int64_t)h.x * CHUNK + h.z;
        finish_long(T, text, N, off, R, h.x, h.y, p, h.w, S, tokc, chunk_cnt, rec_local, pool, counters + 2, pool_cap,
                    err, true);
    }
}

size_t unigram_scratch_bytes(int lane_blocks, int huge_blocks) {
    (void)lane_blocks;  // the long-item kernel works in LDS
    return huge_scratch_bytes() * (size_t)huge_blocks;
}

hipError_t launch_unigram_chunks(const DevTok &T, const uint8_t *text, int64_t N, const uint64_t *off, int64_t R,
                                 const uint32_t *ranges, uint32_t *tokc, uint32_t *chunk_cnt, uint32_t *chunk_ent,
                                 uint32_t *rec_local, const UniWork &W, hipStream_t st) {
    const int64_t n_chunks = (N + CHUNK - 1) / CHUNK;
    if (n_chunks == 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(W.counters, 0, 8 * sizeof(uint32_t), st);  // items, -, pool, huge, items2
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(W.err, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(W.pool, 0, sizeof(uint32_t), st);  // pool word 0: an empty item
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_unigram_chunks, dim3((unsigned)n_chunks), dim3(TOK_THREADS), 0, st, T, text, N, off, R, ranges,
                       tokc, chunk_cnt, chunk_ent, rec_local, W.counters, W.items, W.item_cap, W.err);
    // the narrow jobs' Viterbi and then the long items on st; the wide jobs' Viterbi beside them on W.side
    hipStream_t side = st;
    if (W.side && W.ev_fork && W.ev_join) {
        e = hipEventRecord(W.ev_fork, st);
        if (e == hipSuccess) e = hipStreamWaitEvent(W.side, W.ev_fork, 0);
        if (e != hipSuccess) return e;
        side = W.side;
    }
    hipLaunchKernelGGL(k_unigram_viterbi<false>, dim3((unsigned)n_chunks), dim3(64), 0, st, T, N, off, R, ranges, tokc,
                       chunk_cnt, rec_local);
    hipLaunchKernelGGL(k_unigram_viterbi<true>, dim3((unsigned)n_chunks), dim3(64), 0, side, T, N, off, R, ranges, tokc,
                       chunk_cnt, rec_local);
    // The long items follow the narrow jobs on st: beside the wide jobs, not after them (on
    // held-out text the wide jobs' Viterbi outlasts the narrow one).
    const hipStream_t ls = st;
    // a row's candidate ends: <= Mm + 1 ("▁" row) or <= Mf.  Two stages: items of <= 128
    // normalized bytes (nearly all) with a small LDS footprint and more of them in
    // flight, then the rest (<= 512) from the first stage's overflow list.
    const int g1 = W.lane_blocks * 4 / 3;
#define UNI_LONG_STAGES(KM)                                                                                     \
    hipLaunchKernelGGL((k_unigram_long<KM, LONG_NORM1>), dim3((unsigned)g1), dim3(64), 0, ls, T, text, N, off, R,  \
                       ranges, W.items, W.item_cap, W.counters, W.counters, tokc, chunk_cnt, rec_local, W.pool,      \
                       W.pool_cap, W.items2, W.items2_cap, W.counters + 4, W.err);                                    \
    hipLaunchKernelGGL((k_unigram_long<KM, LONG_NORM>), dim3((unsigned)W.lane_blocks), dim3(64), 0, ls, T, text, N,\
                       off, R, ranges, W.items2, W.items2_cap, W.counters + 4, W.counters, tokc, chunk_cnt,           \
                       rec_local, W.pool, W.pool_cap, W.huge, W.huge_cap, W.counters + 3, W.err);
    if (T.maxlen_meta + 1 <= 20 && T.maxlen_first <= 20) {  // smaller LDS: more items in flight
        UNI_LONG_STAGES(20)
    } else if (T.maxlen_meta + 1 <= 32 && T.maxlen_first <= 32) {
        UNI_LONG_STAGES(32)
    } else {
        UNI_LONG_STAGES(64)
    }
#undef UNI_LONG_STAGES
    hipLaunchKernelGGL(k_unigram_huge, dim3((unsigned)W.huge_blocks), dim3(64), 0, ls, T, text, N, off, R, W.counters,
                       tokc, chunk_cnt, rec_local, W.scratch, W.pool, W.pool_cap, W.huge, W.huge_cap, W.err);
    if (side != st) {
        e = hipEventRecord(W.ev_join, side);
        if (e == hipSuccess) e = hipStreamWaitEvent(st, W.ev_join, 0);
        if (e != hipSuccess) return e;
    }
    return hipGetLastError();
}

}  // namespace sdl
