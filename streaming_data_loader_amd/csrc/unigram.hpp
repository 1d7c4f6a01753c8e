// unigram.hpp -- the t5 tokenizer's per-piece algorithms, written once for the
// host (word-table precompute, assets.cpp) and the gfx950 kernels
// (tokenize_unigram.hip):
//   - UAX #29 extended-grapheme-cluster breaks (crate unicode-segmentation, as
//     tokenizers' Precompiled normalizer uses them: normalizers/precompiled.rs);
//   - the sentencepiece charsmap's shortest-prefix lookup (crate
//     spm_precompiled: DoubleArray::common_prefix_search, results[0]);
//   - Unigram::encode_optimized's Viterbi + fuse_unk (models/unigram/model.rs).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"

namespace sdl {

// ---- grapheme cluster breaks ------------------------------------------------
struct GState {
    uint32_t prev;    // properties of the previous char
    uint32_t ri_odd;  // the RI run ending at prev has odd length
    uint32_t ep_ext;  // prev ends ExtPict Extend*
    uint32_t ep_zwj;  // prev is the ZWJ of ExtPict Extend* ZWJ
    uint32_t incb;    // 1: InCB Consonant [Extend|Linker]*, 2: ... containing a Linker
};

__host__ __device__ inline void gstate_reset(GState &s) {
    s.prev = GB_CONTROL;  // start of text: the first char never joins
    s.ri_odd = s.ep_ext = s.ep_zwj = s.incb = 0;
}

// Is there a cluster boundary before a char with properties p?  Updates s.
__host__ __device__ inline bool gcb_break(GState &s, uint32_t p) {
    const uint32_t a = s.prev & 15u, b = p & 15u;
    const uint32_t ic = (p >> 5) & 3u;
    bool brk;
    if (a == GB_CR && b == GB_LF) brk = false;                                              // GB3
    else if (a == GB_CONTROL || a == GB_CR || a == GB_LF) brk = true;                       // GB4
    else if (b == GB_CONTROL || b == GB_CR || b == GB_LF) brk = true;                       // GB5
    else if (a == GB_L && (b == GB_L || b == GB_V || b == GB_LV || b == GB_LVT)) brk = false;  // GB6
    else if ((a == GB_LV || a == GB_V) && (b == GB_V || b == GB_T)) brk = false;            // GB7
    else if ((a == GB_LVT || a == GB_T) && b == GB_T) brk = false;                          // GB8
    else if (b == GB_EXTEND || b == GB_ZWJ) brk = false;                                    // GB9
    else if (b == GB_SPACING) brk = false;                                                  // GB9a
    else if (a == GB_PREPEND) brk = false;                                                  // GB9b
    else if (ic == 2u && s.incb == 2u) brk = false;                                         // GB9c
    else if (a == GB_ZWJ && s.ep_zwj && (p & GP_EXTPICT)) brk = false;                      // GB11
    else if (a == GB_RI && b == GB_RI && s.ri_odd) brk = false;                             // GB12/13
    else brk = true;                                                                        // GB999
    s.ri_odd = b == GB_RI ? (a == GB_RI ? !s.ri_odd : 1u) : 0u;
    const uint32_t ep_ext = (p & GP_EXTPICT) ? 1u : (b == GB_EXTEND && s.ep_ext) ? 1u : 0u;
    s.ep_zwj = (b == GB_ZWJ && s.ep_ext) ? 1u : 0u;
    s.ep_ext = ep_ext;
    s.incb = ic == 2u ? 1u : (s.incb && ic == 1u) ? 2u : (s.incb && ic == 3u) ? s.incb : 0u;
    s.prev = p;
    return brk;
}

__host__ __device__ inline uint32_t gprop(const uint16_t *page, const uint8_t *block, uint32_t cp) {
    if (cp >= 0x110000u) return 0;
    return block[(uint32_t)page[cp >> 8] * 256u + (cp & 255u)];
}

// ---- charsmap -----------------------------------------------------------------
__host__ __device__ inline uint32_t du_offset(uint32_t u) { return (u >> 10) << ((u & (1u << 9)) >> 6); }

// Offset in the normalized blob of the shortest key that is a prefix of
// bytes [0, n) of `acc`, or -1.  A 0 byte ends the search (spm_precompiled).
template <class Acc>
__host__ __device__ inline int32_t trie_shortest(const uint32_t *units, uint32_t n_units, const Acc &acc, int n) {
    uint32_t pos = du_offset(units[0]);
    for (int i = 0; i < n; ++i) {
        const uint32_t c = acc(i);
        if (c == 0u) return -1;
        pos ^= c;
        if (pos >= n_units) return -1;
        const uint32_t u = units[pos];
        if ((u & ((1u << 31) | 0xFFu)) != c) return -1;
        pos ^= du_offset(u);
        if ((u >> 8) & 1u) return (int32_t)(units[pos] & 0x7FFFFFFFu);
    }
    return -1;
}

// Length of the UTF-8 char with lead byte b (1 for an invalid lead).
__host__ __device__ inline int u8len_lead(uint32_t b) {
    return b < 0x80u ? 1 : (b & 0xE0u) == 0xC0u ? 2 : (b & 0xF0u) == 0xE0u ? 3 : (b & 0xF8u) == 0xF0u ? 4 : 1;
}

// ---- Unigram Viterbi ------------------------------------------------------------
// The piece is bytes [0, n) of `acc`, starting with "▁" (3 bytes).  Nodes are
// byte positions; node e holds the best path ending at e: score (f64), start
// and id.  `cand(s, e, &score)` = id of the vocab piece spelling bytes [s, e)
// (and its score) or -1; s == 0 is the "▁"-prefixed piece.  Candidates are
// visited in tokenizers' order -- starts ascending, then lengths ascending --
// and replace a node only when strictly better.  `maxlen` bounds piece bytes
// (the longest vocab piece; longer substrings cannot be in the trie).
// Writes the ids (fused unk runs looked up whole, else unk_id) in order via
// emit(index, id) and returns their count.
struct UniNode {
    double score;
    int32_t start;  // -1: unset
    int32_t id;
};

// Node e's update by a candidate (st, id, score c): first set, or strictly better.
template <class Nodes>
__host__ __device__ inline void uni_relax(Nodes &nodes, int e, double c, int st, int id) {
    if (nodes.start(e) < 0 || c > nodes.score(e)) nodes.set(e, c, st, id);
}

// Backtrack from node n; consecutive unk nodes fuse into one string, looked
// up whole with cand (models/unigram/model.rs encode_optimized + tokenize).
template <class Cand, class Nodes, class Emit>
__host__ __device__ inline int unigram_backtrack(int n, const Cand &cand, const Nodes &nodes, int unk_id,
                                                 const Emit &emit) {
    int count = 0;
    for (int e = n; e > 0;) {
        const int st = nodes.start(e);
        if (st < 0) break;
        const bool u = nodes.id(e) == unk_id;
        if (!(u && st > 0 && nodes.id(st) == unk_id)) ++count;
        e = st;
    }
    int k = count;
    int run_end = -1;  // end of the unk run being extended leftwards
    for (int e = n; e > 0 && k > 0;) {
        const int st = nodes.start(e);
        if (st < 0) break;
        const bool u = nodes.id(e) == unk_id;
        if (u && st > 0 && nodes.id(st) == unk_id) {  // the run continues leftwards
            if (run_end < 0) run_end = e;
        } else {
            const int end = run_end >= 0 ? run_end : e;
            int id = nodes.id(e);
            if (run_end >= 0 || u) {
                double sc;
                id = cand(st, end, &sc);
                if (id < 0) id = unk_id;
            }
            emit(--k, id);
            run_end = -1;
        }
        e = st;
    }
    return count;
}

template <class Acc, class Cand, class Nodes, class Emit>
__host__ __device__ inline int unigram_viterbi(const Acc &acc, int n, const Cand &cand, Nodes &nodes,
                                               double unk_score, int unk_id, int maxlen, const Emit &emit) {
    if (n <= 0) return 0;
    for (int i = 0; i <= n; ++i) nodes.set(i, 0.0, -1, -1);
    for (int st = 0; st < n;) {
        const int l0 = u8len_lead(acc(st));
        const int mb = l0 < n - st ? l0 : n - st;
        const double base = nodes.score(st);
        bool single = false;
        const int emax = st + maxlen < n ? st + maxlen : n;
        for (int e = st + 1; e <= emax; ++e) {
            if (e < n && (acc(e) & 0xC0u) == 0x80u) continue;  // not a char boundary
            double sc;
            const int id = cand(st, e, &sc);
            if (id < 0) continue;
            uni_relax(nodes, e, sc + base, st, id);
            if (e - st == mb) single = true;
        }
        if (!single) uni_relax(nodes, st + mb, unk_score + base, st, unk_id);
        st += mb;
    }
    return unigram_backtrack(n, cand, nodes, unk_id, emit);
}

// unigram_viterbi over precomputed candidates: rowmask(st) has bit k set when
// the piece ending at e = first_end(st) + k exists (first_end = 3 for the
// "▁" row st == 0, st + 1 otherwise) and at(st, e, &score) returns its id;
// cand(st, e, &score) answers any (st, e) (the fused-unk lookup).  Same visit
// order and result as unigram_viterbi.
template <class Acc, class RowMask, class At, class Cand, class Nodes, class Emit>
__host__ __device__ inline int unigram_viterbi_masked(const Acc &acc, int n, const RowMask &rowmask, const At &at,
                                                      const Cand &cand, Nodes &nodes, double unk_score, int unk_id,
                                                      const Emit &emit) {
    if (n <= 0) return 0;
    for (int i = 0; i <= n; ++i) nodes.set(i, 0.0, -1, -1);
    for (int st = 0; st < n;) {
        const int l0 = u8len_lead(acc(st));
        const int mb = l0 < n - st ? l0 : n - st;
        const double base = nodes.score(st);
        const int fe = st == 0 ? 3 : st + 1;
        uint64_t m = rowmask(st);
        const bool single = (m >> (st + mb - fe)) & 1ull;
        while (m) {
            const int k = __builtin_ctzll(m);
            m &= m - 1;
            const int e = fe + k;
            double sc;
            const int id = at(st, e, &sc);
            uni_relax(nodes, e, sc + base, st, id);
        }
        if (!single) uni_relax(nodes, st + mb, unk_score + base, st, unk_id);
        st += mb;
    }
    return unigram_backtrack(n, cand, nodes, unk_id, emit);
}

}  // namespace sdl
