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
// Words are found on the raw bytes.  A *simple* word -- printable ASCII only,
// bounded by ASCII whitespace, a record edge or an added token -- is its own
// normalization (its clusters are single ASCII chars and the charsmap keeps
// printable ASCII; checked on the host), so its ids are Viterbi("▁" + word):
//   1. one probe of the word table (vocab "▁w" pieces with their precomputed
//      Viterbi ids) settles most words;
//   2. misses run the Viterbi lane-per-word, DP nodes in LDS, every candidate
//      piece one cuckoo probe of the vocab table.
// Every other word (non-ASCII or control bytes, > UNI_WMAX bytes, running past
// the window) is a *long item*: its chunk entry is a marker and k_unigram_long
// normalizes it (grapheme clusters, trie), splits, and runs the Viterbi per
// piece, lane per item, writing its ids to a pool the compaction expands.
// Items whose normalized text exceeds a lane's scratch go to k_unigram_huge.
#include "common.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "tok_device.hpp"
#include "unigram.hpp"

namespace sdl {

namespace {

enum : uint8_t { U_WS = 0, U_P = 1, U_X = 2, U_SPEC = 3, U_SPX = 4 };
constexpr uint32_t LMARK = 0x80000000u, LPEND = 0x40000000u;
__device__ const uint8_t kMetaBytes[3] = {0xE2, 0x96, 0x81};

typedef __attribute__((address_space(3))) double lds_f64;

__device__ __forceinline__ uint32_t uni_ascii(uint32_t b) {
    if (b == 32u || b == 9u || b == 10u || b == 12u || b == 13u) return U_WS;
    if (b - 0x21u < 0x5Eu) return U_P;
    return U_X;
}
__device__ __forceinline__ bool ascii_ws(uint32_t b) { return b == 32u || b == 9u || b == 10u || b == 12u || b == 13u; }

// id of the slot (payload bytes acc(start .. start+n), cont) or -1: exact
template <class Acc>
__device__ int probe_acc(const DevTok &T, const Acc &acc, int start, int n, uint32_t cont) {
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
    const Probe P = probe_load(T, h);
    for (int which = 0; which < 2; ++which) {
        const uint4 a = which ? P.a2 : P.a1, b = which ? P.b2 : P.b1;
        if (!slot_match(a, b, key, first)) continue;
        bool ok = true;
        for (int k = 16; k < n && ok; ++k) ok = T.vpool[a.z + k] == acc(start + k);
        if (ok) return (int32_t)a.y;
    }
    return -1;
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

// ---- long items: normalize, split, Viterbi (one lane, sequential) ------------
struct Scratch {
    uint8_t *nb;     // normalized bytes
    UniNode *nodes;  // Viterbi nodes
    uint32_t *ids;   // ids of the item
    int cap;         // normalized byte capacity (ids: 2 * cap + 8, nodes: cap + 8)
};

// strict UTF-8 decode as oracle/orc_unigram.c (u8len): raw length consumed,
// cp, the sanitized bytes (invalid -> U+FFFD) and their count
__device__ __forceinline__ int dec_char(const uint8_t *t, int64_t q, int64_t end, uint32_t *cp, uint32_t *bytes,
                                        int *blen) {
    const uint32_t b = t[q];
    if (b < 0x80u) {
        *cp = b;
        *bytes = b;
        *blen = 1;
        return 1;
    }
    int len;
    uint32_t c, mn;
    if ((b & 0xE0u) == 0xC0u) { len = 2; c = b & 0x1Fu; mn = 0x80u; }
    else if ((b & 0xF0u) == 0xE0u) { len = 3; c = b & 0x0Fu; mn = 0x800u; }
    else if ((b & 0xF8u) == 0xF0u) { len = 4; c = b & 0x07u; mn = 0x10000u; }
    else len = 0;
    bool ok = len > 0 && q + len <= end;
    uint32_t raw = b;
    for (int k = 1; ok && k < len; ++k) {
        const uint32_t x = t[q + k];
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

// Precompiled::normalize of raw word [a, b); ctx_space: the byte before a is
// ' ' (so a cluster may run on from it: such chars are looked up one by one,
// as the whole cluster -- which starts with ' ' -- matches no key).  Returns the
// normalized length, or -1 when it exceeds cap.
__device__ int normalize_word(const DevTok &T, const uint8_t *text, int64_t a, int64_t b, bool ctx_space, uint8_t *nb,
                              int cap) {
    GState g;
    gstate_reset(g);
    if (ctx_space) gcb_break(g, gprop(T.tpage, T.tblock, 0x20u));
    int nl = 0;
    bool ovf = false;
    auto put_bytes = [&](uint32_t bytes, int n) {
        if (nl + n > cap) { ovf = true; return; }
        for (int k = 0; k < n; ++k) nb[nl + k] = (uint8_t)(bytes >> (8 * k));
        nl += n;
    };
    auto put_norm = [&](int32_t off) {
        for (uint32_t i = (uint32_t)off; i < T.tnorm_len && T.tnorm[i]; ++i) {
            if (nl >= cap) { ovf = true; return; }
            nb[nl++] = T.tnorm[i];
        }
    };
    bool first = true;
    int64_t q = a;
    while (q < b && !ovf) {
        const int64_t cs = q;
        uint32_t cp, bytes;
        int bl;
        q += dec_char(text, q, b, &cp, &bytes, &bl);
        const bool brk = gcb_break(g, gprop(T.tpage, T.tblock, cp));
        const bool forced = first && ctx_space && !brk;
        first = false;
        uint32_t buf0 = bytes, buf1 = 0;  // the cluster's first 8 sanitized bytes
        int L = bl;
        while (q < b) {
            uint32_t cp2, by2;
            int bl2;
            const int rl = dec_char(text, q, b, &cp2, &by2, &bl2);
            GState g2 = g;
            if (gcb_break(g2, gprop(T.tpage, T.tblock, cp2))) break;
            g = g2;
            for (int k = 0; k < bl2; ++k, ++L) {
                const uint32_t v = (by2 >> (8 * k)) & 0xFFu;
                if (L < 4) buf0 |= v << (8 * L);
                else if (L < 8) buf1 |= v << (8 * (L - 4));
            }
            q += rl;
        }
        if (!forced && L < 6) {
            const int32_t r = trie_shortest(T.trie, T.trie_units, [&](int i) -> uint32_t {
                return i < 4 ? (buf0 >> (8 * i)) & 0xFFu : (buf1 >> (8 * (i - 4))) & 0xFFu;
            }, L);
            if (r >= 0) {
                put_norm(r);
                continue;
            }
        }
        for (int64_t x = cs; x < q && !ovf;) {  // per char
            uint32_t c3, b3;
            int l3;
            x += dec_char(text, x, b, &c3, &b3, &l3);
            const int32_t r = trie_shortest(T.trie, T.trie_units,
                                            [&](int i) -> uint32_t { return (b3 >> (8 * i)) & 0xFFu; }, l3);
            if (r >= 0) put_norm(r);
            else put_bytes(b3, l3);
        }
    }
    return ovf ? -1 : nl;
}

struct GNodes {
    UniNode *v;
    __device__ void set(int i, double s, int st, int id) const { v[i] = UniNode{s, st, id}; }
    __device__ double score(int i) const { return v[i].score; }
    __device__ int start(int i) const { return v[i].start; }
    __device__ int id(int i) const { return v[i].id; }
};

// WhitespaceSplit + Metaspace + Unigram over nb[0, nl); ids -> S.ids.
// Returns the id count (or -1 if the ids exceed their capacity).
__device__ int tokenize_normalized(const DevTok &T, const Scratch &S, int nl) {
    const uint8_t *nb = S.nb;
    int k = 0;
    const int idcap = 2 * S.cap + 8;
    auto ws_at = [&](int i, int *len) {
        const uint32_t b = nb[i];
        uint32_t cp = b;
        int l = u8len_lead(b);
        if (l > 1) {
            cp = b & (l == 2 ? 0x1Fu : l == 3 ? 0x0Fu : 0x07u);
            for (int j = 1; j < l; ++j) cp = cp << 6 | (nb[i + j] & 0x3Fu);
        }
        *len = l;
        return (gprop(T.tpage, T.tblock, cp) & GP_WS) != 0u;
    };
    int i = 0;
    while (i < nl) {
        int l;
        if (ws_at(i, &l)) { i += l; continue; }
        int j = i;
        while (j < nl && !ws_at(j, &l)) j += l;
        // word [i, j): pieces start at i and before every "▁"; a word not
        // starting with "▁" gets one prepended (Metaspace, add_prefix_space)
        int ps = i;
        bool virt = !(j - i >= 3 && nb[i] == 0xE2 && nb[i + 1] == 0x96 && nb[i + 2] == 0x81);
        for (int t = i + 1; t <= j; ++t) {
            const bool cut = t == j || (t + 3 <= j && nb[t] == 0xE2 && nb[t + 1] == 0x96 && nb[t + 2] == 0x81);
            if (!cut) continue;
            const int off = virt ? 3 : 0;
            const int n = t - ps + off;
            auto acc = [&](int x) -> uint32_t { return x < off ? kMetaBytes[x] : nb[ps + x - off]; };
            auto probe = [&](int s, int e) -> int {
                if (s == 0) return (e - 3 <= T.maxlen_meta) ? probe_acc(T, acc, 3, e - 3, UC_META) : -1;
                return (e - s <= T.maxlen_first) ? probe_acc(T, acc, s, e - s, UC_PIECE) : -1;
            };
            if (k + n + 1 > idcap) return -1;
            GNodes nodes{S.nodes};
            const int base = k;
            k += unigram_viterbi(acc, n, probe, nodes, T.uscore, T.unk_score, T.unk_id, T.maxlen_piece,
                                 [&](int x, int id) { S.ids[base + x] = (uint32_t)id; });
            ps = t;
            virt = false;
        }
        i = j;
    }
    return k;
}


// Per-lane LDS nodes of the chunk kernel (node-major: conflict-free)
struct LdsNodes {
    lds_f64 *sc;
    lds_u32 *bp;
    int lane;
    __device__ void set(int i, double s, int st, int id) const {
        sc[i * 64 + lane] = s;
        bp[i * 64 + lane] = (uint32_t)(st & 0xFFFF) | ((uint32_t)(id & 0xFFFF) << 16);
    }
    __device__ double score(int i) const { return sc[i * 64 + lane]; }
    __device__ int start(int i) const {
        const uint32_t v = bp[i * 64 + lane] & 0xFFFFu;
        return v == 0xFFFFu ? -1 : (int)v;
    }
    __device__ int id(int i) const {
        const uint32_t v = bp[i * 64 + lane] >> 16;
        return v == 0xFFFFu ? -1 : (int)v;
    }
};

}  // namespace

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(TOK_THREADS) void k_unigram_chunks(
    DevTok T, const uint8_t *__restrict__ text, int64_t N, const uint64_t *__restrict__ off, int64_t R,
    const uint32_t *__restrict__ ranges, uint32_t *__restrict__ tokc, uint32_t *__restrict__ chunk_cnt,
    uint32_t *__restrict__ chunk_ent, uint32_t *__restrict__ rec_local, uint32_t *__restrict__ long_count,
    uint32_t *__restrict__ lchunks, uint32_t *__restrict__ lchunk_count) {
    __shared__ __attribute__((aligned(16))) uint8_t s_win[WIN + 32];
    __shared__ __attribute__((aligned(16))) uint8_t s_cls[WIN];
    __shared__ uint32_t s_rbits[RBITS_WORDS + 1];
    __shared__ uint16_t s_pieces[CHUNK + 1];  // prel | SPEC << 12
    __shared__ uint16_t s_plen[CHUNK];        // piece length, 0 = runs past the window; bit 15: simple
    __shared__ uint16_t s_stage[2 * CHUNK + 64];  // ids staged at 2 * prel
    __shared__ uint16_t s_cnt[CHUNK];
    __shared__ uint16_t s_poff[CHUNK];
    __shared__ uint16_t s_rb[RB_CAP];
    __shared__ uint32_t s_scratch[8];
    __shared__ double s_nsc[UNI_NODES * 64];
    __shared__ uint32_t s_nbp[UNI_NODES * 64];

    const int tid = threadIdx.x;
    const int lane = tid;
    const int64_t c0 = (int64_t)blockIdx.x * CHUNK;
    const int64_t c1 = c0 + CHUNK < N ? c0 + CHUNK : N;
    const int64_t w0 = c0 - HALO_L;
    const lds_u8 *win = (const lds_u8 *)s_win;
    lds_u8 *cls = (lds_u8 *)s_cls;
    const lds_u32 *rbits = (const lds_u32 *)s_rbits;

    // ---- 1. load + classify ----------------------------------------------------
    const uint4 v = load16(text, c0 + 16 * tid, N);
    *reinterpret_cast<uint4 *>(s_win + HALO_L + 16 * tid) = v;
    uint4 hv = make_uint4(0, 0, 0, 0);
    int64_t hp = 0;
    if (tid < (WIN - CHUNK) / 16) {
        hp = tid < HALO_L / 16 ? w0 + 16 * tid : c0 + CHUNK + 16 * (tid - HALO_L / 16);
        hv = load16(text, hp, N);
        *reinterpret_cast<uint4 *>(s_win + (hp - w0)) = hv;
    }
    if (tid < 2) *reinterpret_cast<uint4 *>(s_win + WIN + 16 * tid) = make_uint4(0, 0, 0, 0);
    if (tid <= RBITS_WORDS) s_rbits[tid] = 0;
    const int64_t ra = ranges[3 * blockIdx.x], rz = ranges[3 * blockIdx.x + 1], r_lo = ranges[3 * blockIdx.x + 2];
    const int nrb = (int)(rz - ra);
    const bool rb_ok = nrb <= RB_CAP;
    if (tid == 0) s_scratch[0] = s_scratch[1] = s_scratch[2] = 0;
    __syncthreads();
    for (int k = tid; k < nrb; k += TOK_THREADS) {
        const int rel = (int)((int64_t)off[ra + k] - w0);
        atomicOr(&s_rbits[rel >> 5], 1u << (rel & 31));
        if (rb_ok) s_rb[k] = (uint16_t)rel;
    }
    auto classify16 = [&](const uint4 &x, int wi0) {
        const uint32_t wv[4] = {x.x, x.y, x.z, x.w};
        uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < 16; ++i) o[i >> 2] |= uni_ascii((wv[i >> 2] >> (8 * (i & 3))) & 0xFFu) << (8 * (i & 3));
        *reinterpret_cast<uint4 *>(s_cls + wi0) = make_uint4(o[0], o[1], o[2], o[3]);
    };
    classify16(v, HALO_L + 16 * tid);
    if (tid < (WIN - CHUNK) / 16) classify16(hv, (int)(hp - w0));
    __syncthreads();

    const Ctx C{&T, win, rbits, w0, text, N, off, R};
    auto cbyte = [&](int64_t q) -> uint32_t { return C.byte(q); };
    auto cbnd = [&](int64_t q) -> bool { return C.rstart(q); };
    // added tokens (override the classes of their bytes)
    if (T.n_special) {
        for (int wi = tid; wi < WIN; wi += TOK_THREADS) {
            const int64_t p = w0 + wi;
            if (win[wi] != (uint8_t)'<' || p < 0 || p >= N) continue;
            int l = 0;
            if (uni_special(T, p, N, cbyte, cbnd, &l) < 0) continue;
            cls[wi] = U_SPEC;
            for (int j = 1; j < l && wi + j < WIN; ++j) cls[wi + j] = U_SPX;
        }
        __syncthreads();
    }

    // ---- 2. piece starts: added tokens, and the first byte of every word ------
    const int64_t s0 = c0 + 16 * tid;
    const int nown = s0 >= c1 ? 0 : (int)(c1 - s0 < 16 ? c1 - s0 : 16);
    uint32_t pmask = 0;
    for (int i = 0; i < nown; ++i) {
        const int wi = HALO_L + 16 * tid + i;
        const uint32_t k = cls[wi];
        if (k == U_SPEC) { pmask |= 1u << i; continue; }
        if (k != U_P && k != U_X) continue;
        const uint32_t pk = cls[wi - 1];
        if (pk == U_WS || pk == U_SPX || pk == U_SPEC || ((rbits[wi >> 5] >> (wi & 31)) & 1u)) pmask |= 1u << i;
    }
    uint32_t np_total;
    uint32_t pbase = block_excl_sum<TOK_THREADS>((uint32_t)__builtin_popcount(pmask), &np_total, s_scratch + 4);
    for (uint32_t m = pmask; m;) {
        const int i = __builtin_ctz(m);
        m &= m - 1;
        const int wi = HALO_L + 16 * tid + i;
        s_pieces[pbase++] = (uint16_t)((16 * tid + i) | (cls[wi] == U_SPEC ? 1u << 12 : 0u));
    }
    __syncthreads();
    const int np = (int)np_total;

    // ---- 3. per piece: length, then word table / added token / long item -------
    lds_u16 *stage = (lds_u16 *)s_stage;
    lds_u16 *cnt = (lds_u16 *)s_cnt;
    uint16_t *s_pend = s_poff;  // misses for the Viterbi (s_poff is free until step 5)
    const lds_u32 *w32 = (const lds_u32 *)s_win;
    for (int pi = tid; pi < np; pi += TOK_THREADS) {
        const uint32_t pc = s_pieces[pi];
        const int prel = (int)(pc & 0xFFFu);
        const int wi0 = HALO_L + prel;
        bool pend = false;
        if (pc & (1u << 12)) {
            int l = 0;
            const int id = uni_special(T, c0 + prel, N, cbyte, cbnd, &l);
            stage[2 * prel] = (uint16_t)(id < 0 ? T.unk_id : id);
            cnt[pi] = 1;
            s_plen[pi] = (uint16_t)l;
        } else {
            // word end: first whitespace / added token / record start / text end
            int wi = wi0 + 1;
            bool simple = cls[wi0] == U_P;
            int len = 0;
            for (;; ++wi) {
                if (wi >= WIN - 8) { len = 0; break; }  // runs past the window
                if (w0 + wi >= N) { len = wi - wi0; break; }
                const uint32_t k = cls[wi];
                if (k == U_WS || k == U_SPEC || ((rbits[wi >> 5] >> (wi & 31)) & 1u)) { len = wi - wi0; break; }
                simple = simple && k == U_P;
            }
            s_plen[pi] = (uint16_t)len;
            if (simple && len > 0 && len <= UNI_WMAX) {
                int packed;
                if (len <= 16) {
                    const int a = wi0 >> 2;
                    const uint32_t sh = (uint32_t)(wi0 & 3);
                    const uint32_t x0 = w32[a], x1 = w32[a + 1], x2 = w32[a + 2], x3 = w32[a + 3], x4 = w32[a + 4];
                    const W16 raw{__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh),
                                  __builtin_amdgcn_alignbyte(x3, x2, sh), __builtin_amdgcn_alignbyte(x4, x3, sh)};
                    const W16 w = keep_bytes(raw, len);
                    packed = probe_result(probe_load(T, hash16(w, (uint32_t)len, UC_WORD)),
                                          (uint32_t)len | (UC_WORD << 8), w);
                } else {
                    packed = probe_acc(T, [&](int i) -> uint32_t { return win[wi0 + i]; }, 0, len, UC_WORD);
                }
                if (packed >= 0) {
                    const int k = packed >> 24;
                    const uint32_t x = (uint32_t)packed & 0xFFFFFFu;
                    if (k == 1) stage[2 * prel] = (uint16_t)x;
                    else
                        for (int j = 0; j < k; ++j) stage[2 * prel + j] = T.wres[x + j];
                    cnt[pi] = (uint16_t)k;
                } else {
                    pend = true;
                }
            } else {
                // long item: marker (2 stage slots); finished by k_unigram_long
                const uint32_t mk = LMARK | LPEND | ((uint32_t)(len > 0xFFFFF ? 0 : len) << 10) | (uint32_t)prel;
                stage[2 * prel] = (uint16_t)(mk & 0xFFFFu);
                stage[2 * prel + 1] = (uint16_t)(mk >> 16);
                cnt[pi] = 0xFFFFu;
                atomicAdd(long_count, 1u);
                s_scratch[2] = 1u;
            }
        }
        const uint64_t pm = __ballot(pend);
        if (pm) {
            const int leader = __builtin_ctzll(pm);
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(&s_scratch[1], (uint32_t)__popcll(pm));
            base = __shfl(base, leader, 64);
            if (pend) s_pend[base + __popcll(pm & ((1ull << lane) - 1ull))] = (uint16_t)pi;
        }
    }
    __syncthreads();

    // ---- 4. Viterbi of the word-table misses, lane per word -----------------------
    const int npend = (int)s_scratch[1];
    const LdsNodes nodes{(lds_f64 *)s_nsc, (lds_u32 *)s_nbp, lane};
    for (int q = lane; q < npend; q += 64) {
        const int pi = s_pend[q];
        const int prel = (int)(s_pieces[pi] & 0xFFFu);
        const int len = s_plen[pi];
        const int wi0 = HALO_L + prel;
        auto acc = [&](int i) -> uint32_t { return i < 3 ? kMetaBytes[i] : (uint32_t)win[wi0 + i - 3]; };
        auto probe = [&](int s, int e) -> int {
            // payload = word bytes [ws, ws + n) with cont META (s == 0) or PIECE
            const int ws = s == 0 ? 0 : s - 3;
            const int n = s == 0 ? e - 3 : e - s;
            const uint32_t cont = s == 0 ? UC_META : UC_PIECE;
            if (n > (s == 0 ? T.maxlen_meta : T.maxlen_first)) return -1;
            if (n <= 16) {
                const int b = wi0 + ws;
                const int a = b >> 2;
                const uint32_t sh = (uint32_t)(b & 3);
                const uint32_t x0 = w32[a], x1 = w32[a + 1], x2 = w32[a + 2], x3 = w32[a + 3], x4 = w32[a + 4];
                const W16 raw{__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh),
                              __builtin_amdgcn_alignbyte(x3, x2, sh), __builtin_amdgcn_alignbyte(x4, x3, sh)};
                const W16 w = keep_bytes(raw, n);
                return probe_result(probe_load(T, hash16(w, (uint32_t)n, cont)), (uint32_t)n | (cont << 8), w);
            }
            return probe_acc(T, [&](int i) -> uint32_t { return win[wi0 + i]; }, ws, n, cont);
        };
        const int k = unigram_viterbi(acc, len + 3, probe, nodes, T.uscore, T.unk_score, T.unk_id, T.maxlen_piece,
                                      [&](int x, int id) { stage[2 * prel + x] = (uint16_t)id; });
        cnt[pi] = (uint16_t)k;
    }
    __syncthreads();

    // ---- 5. compact ids into this chunk's tokc slice ------------------------------
    const int per = (np + TOK_THREADS - 1) / TOK_THREADS;
    const int a0 = tid * per < np ? tid * per : np;
    const int a1 = a0 + per < np ? a0 + per : np;
    uint32_t mine = 0;
    for (int i = a0; i < a1; ++i) mine += s_cnt[i] == 0xFFFFu ? 1u : s_cnt[i];
    uint32_t total;
    uint32_t base = block_excl_sum<TOK_THREADS>(mine, &total, s_scratch + 4);
    uint32_t *dst = tokc + (int64_t)blockIdx.x * UNI_STAGE;
    for (int i = a0; i < a1; ++i) {
        s_poff[i] = (uint16_t)base;
        const int prel = s_pieces[i] & 0xFFF;
        const int k = s_cnt[i];
        if (k == 0xFFFF) {
            dst[base++] = (uint32_t)s_stage[2 * prel] | ((uint32_t)s_stage[2 * prel + 1] << 16);
            continue;
        }
        for (int j = 0; j < k; ++j) dst[base + j] = s_stage[2 * prel + j];
        base += k;
    }
    __syncthreads();
    if (tid == 0) {
        chunk_cnt[blockIdx.x] = chunk_ent[blockIdx.x] = total;
        if (s_scratch[2]) lchunks[atomicAdd(lchunk_count, 1u)] = (uint32_t)blockIdx.x;
    }
    const int k_lo = (int)(r_lo - ra);
    for (int k = k_lo + tid;; k += TOK_THREADS) {
        int64_t pos;
        if (rb_ok) {
            if (k >= nrb) break;
            pos = w0 + s_rb[k];
        } else {
            if (ra + k > R) break;
            pos = (int64_t)off[ra + k];
        }
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

namespace {

// Finishes long item (chunk c, entry e, raw start p, raw length len or 0):
// returns false when its normalized text exceeds S.cap (nothing written).
__device__ bool finish_long(const DevTok &T, const uint8_t *text, int64_t N, const uint64_t *off, int64_t R,
                            uint32_t c, uint32_t e, int64_t p, int64_t len, const Scratch &S, uint32_t *tokc,
                            uint32_t *chunk_cnt, uint32_t *rec_local, uint32_t *pool, uint32_t *pool_count,
                            uint32_t pool_cap, uint32_t *err, bool last_resort) {
    // record containing p
    int64_t lo = 0, hi = R;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int64_t)off[mid + 1] <= p) lo = mid + 1; else hi = mid;
    }
    const int64_t rec = lo, rs = (int64_t)off[rec], re = (int64_t)off[rec + 1] < N ? (int64_t)off[rec + 1] : N;
    int64_t end = p + len;
    if (len == 0) {  // ran past its chunk's window: scan to the word's end
        auto byte = [&](int64_t q) -> uint32_t { return text[q]; };
        auto bnd = [&](int64_t q) -> bool { return q >= re; };
        for (end = p + 1; end < re; ++end) {
            const uint32_t b = text[end];
            if (ascii_ws(b)) break;
            int l;
            if (b == (uint32_t)'<' && T.n_special && uni_special(T, end, N, byte, bnd, &l) >= 0) break;
        }
    }
    const bool ctx_space = p > rs && text[p - 1] == (uint8_t)' ';
    const int nl = normalize_word(T, text, p, end, ctx_space, S.nb, S.cap);
    int k = 0;
    if (nl < 0) {
        if (!last_resort) return false;
        atomicOr(err, 16u);  // a whitespace-free run beyond UNI_HUGE_NORM normalized bytes: dropped
    } else {
        k = tokenize_normalized(T, S, nl);
        if (k < 0) {
            atomicOr(err, 2u);
            k = 0;
        }
    }
    // pool word 0 is an empty item; allocations start at 1
    const uint32_t at = 1u + atomicAdd(pool_count, (uint32_t)k + 1u);
    if ((uint64_t)at + (uint32_t)k + 1u > pool_cap) {
        atomicOr(err, 4u);
        k = 0;
        tokc[(int64_t)c * UNI_STAGE + e] = LMARK;  // an empty item (pool slot 0 holds 0)
    } else {
        pool[at] = (uint32_t)k;
        for (int j = 0; j < k; ++j) pool[at + 1 + j] = S.ids[j];
        tokc[(int64_t)c * UNI_STAGE + e] = LMARK | at;
    }
    const uint32_t extra = (uint32_t)k - 1u;  // the entry counted one id
    if (extra) {
        atomicAdd(&chunk_cnt[c], extra);
        const int64_t cend = ((int64_t)c + 1) * CHUNK;
        for (int64_t r = rec + 1; r < R && (int64_t)off[r] < cend; ++r)
            if ((int64_t)off[r] > p) atomicAdd(&rec_local[r], extra);
    }
    return true;
}

}  // namespace

// Long items, lane per item, per chunk of the lchunks list.
__global__ __launch_bounds__(64) void k_unigram_long(DevTok T, const uint8_t *__restrict__ text, int64_t N,
                                                     const uint64_t *__restrict__ off, int64_t R,
                                                     const uint32_t *__restrict__ lchunks,
                                                     const uint32_t *__restrict__ lchunk_count,
                                                     const uint32_t *__restrict__ chunk_ent, uint32_t *tokc,
                                                     uint32_t *chunk_cnt, uint32_t *rec_local, uint8_t *scratch,
                                                     uint32_t *pool, uint32_t *pool_count, uint32_t pool_cap,
                                                     uint4 *huge, uint32_t *huge_count, uint32_t huge_cap,
                                                     uint32_t *err) {
    const int lane = lane_id();
    const size_t per = (size_t)UNI_LANE_NORM + sizeof(UniNode) * (UNI_LANE_NORM + 8) + 4 * (2 * UNI_LANE_NORM + 8);
    uint8_t *mine = scratch + ((size_t)blockIdx.x * 64 + lane) * per;
    const Scratch S{mine + sizeof(UniNode) * (UNI_LANE_NORM + 8) + 4 * (2 * UNI_LANE_NORM + 8),
                    reinterpret_cast<UniNode *>(mine),
                    reinterpret_cast<uint32_t *>(mine + sizeof(UniNode) * (UNI_LANE_NORM + 8)), UNI_LANE_NORM};
    const uint32_t nl = *lchunk_count;
    for (uint32_t i = blockIdx.x; i < nl; i += gridDim.x) {
        const uint32_t c = lchunks[i];
        const uint32_t ne = chunk_ent[c];
        for (uint32_t e0 = 0; e0 < ne; e0 += 64) {
            const uint32_t e = e0 + lane;
            const uint32_t x = e < ne ? tokc[(int64_t)c * UNI_STAGE + e] : 0u;
            if ((x & (LMARK | LPEND)) != (LMARK | LPEND)) continue;
            const int64_t p = (int64_t)c * CHUNK + (x & 0x3FFu);
            const int64_t len = (x >> 10) & 0xFFFFFu;
            if (!finish_long(T, text, N, off, R, c, e, p, len, S, tokc, chunk_cnt, rec_local, pool, pool_count,
                             pool_cap, err, false)) {
                const uint32_t h = atomicAdd(huge_count, 1u);
                if (h < huge_cap) huge[h] = make_uint4(c, e, (uint32_t)(x & 0x3FFu), (uint32_t)len);
                else atomicOr(err, 8u);
            }
        }
    }
}

// Items whose normalized text exceeds a lane's scratch: one wave each, lane 0.
__global__ __launch_bounds__(64) void k_unigram_huge(DevTok T, const uint8_t *__restrict__ text, int64_t N,
                                                     const uint64_t *__restrict__ off, int64_t R, uint32_t *tokc,
                                                     uint32_t *chunk_cnt, uint32_t *rec_local, uint8_t *scratch,
                                                     uint32_t *pool, uint32_t *pool_count, uint32_t pool_cap,
                                                     const uint4 *huge, const uint32_t *huge_count, uint32_t huge_cap,
                                                     uint32_t *err) {
    if (lane_id() != 0) return;
    const size_t per = (size_t)UNI_HUGE_NORM + sizeof(UniNode) * (UNI_HUGE_NORM + 8) + 4 * (2 * UNI_HUGE_NORM + 8);
    uint8_t *mine = scratch + (size_t)blockIdx.x * per;
    const Scratch S{mine + sizeof(UniNode) * (UNI_HUGE_NORM + 8) + 4 * (2 * UNI_HUGE_NORM + 8),
                    reinterpret_cast<UniNode *>(mine),
                    reinterpret_cast<uint32_t *>(mine + sizeof(UniNode) * (UNI_HUGE_NORM + 8)), UNI_HUGE_NORM};
    uint32_t nh = *huge_count;
    if (nh > huge_cap) nh = huge_cap;
    for (uint32_t i = blockIdx.x; i < nh; i += gridDim.x) {
        const uint4 h = huge[i];
        const int64_t p = (int64_t)h.x * CHUNK + h.z;
        finish_long(T, text, N, off, R, h.x, h.y, p, h.w, S, tokc, chunk_cnt, rec_local, pool, pool_count, pool_cap,
                    err, true);
    }
}

size_t unigram_scratch_bytes(int lane_blocks, int huge_blocks) {
    const size_t lane = (size_t)UNI_LANE_NORM + sizeof(UniNode) * (UNI_LANE_NORM + 8) + 4 * (2 * UNI_LANE_NORM + 8);
    const size_t huge = (size_t)UNI_HUGE_NORM + sizeof(UniNode) * (UNI_HUGE_NORM + 8) + 4 * (2 * UNI_HUGE_NORM + 8);
    return lane * 64 * (size_t)lane_blocks + huge * (size_t)huge_blocks;
}

hipError_t launch_unigram_chunks(const DevTok &T, const uint8_t *text, int64_t N, const uint64_t *off, int64_t R,
                                 const uint32_t *ranges, uint32_t *tokc, uint32_t *chunk_cnt, uint32_t *chunk_ent,
                                 uint32_t *rec_local, const UniWork &W, hipStream_t st) {
    const int64_t n_chunks = (N + CHUNK - 1) / CHUNK;
    if (n_chunks == 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(W.counters, 0, 4 * sizeof(uint32_t), st);  // long, lchunk, pool, huge
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(W.err, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_unigram_chunks, dim3((unsigned)n_chunks), dim3(TOK_THREADS), 0, st, T, text, N, off, R, ranges,
                       tokc, chunk_cnt, chunk_ent, rec_local, W.counters + 0, W.lchunks, W.counters + 1);
    // pool word 0 stays 0 (an empty item); items allocate after it
    e = hipMemsetAsync(W.pool, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_unigram_long, dim3((unsigned)W.lane_blocks), dim3(64), 0, st, T, text, N, off, R, W.lchunks,
                       W.counters + 1, chunk_ent, tokc, chunk_cnt, rec_local, W.scratch, W.pool, W.counters + 2,
                       W.pool_cap, W.huge, W.counters + 3, W.huge_cap, W.err);
    hipLaunchKernelGGL(k_unigram_huge, dim3((unsigned)W.huge_blocks), dim3(64), 0, st, T, text, N, off, R, tokc,
                       chunk_cnt, rec_local, W.scratch + (size_t)W.lane_blocks * 64 *
                           ((size_t)UNI_LANE_NORM + sizeof(UniNode) * (UNI_LANE_NORM + 8) + 4 * (2 * UNI_LANE_NORM + 8)),
                       W.pool, W.counters + 2, W.pool_cap, W.huge, W.counters + 3, W.huge_cap, W.err);
    return hipGetLastError();
}

}  // namespace sdl
