// tokenize_wordpiece.hip -- BERT WordPiece tokenization of a text arena on gfx950.
//
// Restates, for a whole arena of records at once, what the reference does one
// record at a time in TokenizerHolder::get_ids -> tokenizers::Tokenizer::encode
// (rust/src/tokenizer/tokenizer_holder.rs:19-28; crate tokenizers 0.13.1):
//   AddedVocabulary split (raw-text match of the added tokens)
//   -> BertNormalizer (clean_text, CJK padding, NFD + strip Mn, lowercase)
//   -> BertPreTokenizer (split on whitespace, isolate punctuation)
//   -> WordPiece (greedy longest-match-first, "##" continuation, 100-char cap).
// The template's [CLS]/[SEP] and the wrapper's framing are added at row
// assembly (rows.hip).
//
// One 256-thread workgroup owns CHUNK = 4096 bytes of the arena:
//   1. stage [c0-16, c0+4096+240) in LDS with 16-B coalesced loads;
//   2. each thread classifies its 16 bytes (ASCII from an LDS table, the rest
//      through the two-level Unicode table in L2) into visible classes;
//   3. a block scan carries "last visible class" across threads, so every
//      thread knows where pieces (words, isolated chars, added tokens) start;
//   4. piece starts are compacted into an LDS list (block prefix sum);
//   5. each thread WordPiece-tokenizes pieces i, i+256, ... reading the word
//      from LDS and probing the vocab hash (32-B slots, L2-resident); tokens of
//      a piece starting at byte p are staged at stage[p-c0] (a piece never has
//      more tokens than bytes, so these never collide);
//   6. a second block scan compacts the staged tokens into this chunk's region
//      of `tokc` and records where each record boundary falls.
#include "common.hpp"
#include "device_util.hpp"
#include "kernels.hpp"

namespace sdl {

namespace {

struct Src {
    const uint8_t *win;    // LDS copy of [w0, w0 + WIN)
    const uint8_t *rflag;  // LDS: 1 where a record starts, same window
    int64_t w0;
    const uint8_t *text;
    int64_t N;
    const uint64_t *off;   // record offsets, R+1 entries
    int64_t R;

    __device__ __forceinline__ bool in_win(int64_t p) const { return (uint64_t)(p - w0) < (uint64_t)WIN; }
    __device__ __forceinline__ uint32_t byte(int64_t p) const { return in_win(p) ? win[p - w0] : text[p]; }
    // true when a record starts at p (p in [0, N])
    __device__ bool rstart(int64_t p) const {
        if (in_win(p)) return rflag[p - w0] != 0;
        int64_t lo = 0, hi = R;  // any off[r] == p ?
        while (lo < hi) {
            int64_t mid = (lo + hi) >> 1;
            if ((int64_t)off[mid] < p) lo = mid + 1; else hi = mid;
        }
        return lo <= R && (int64_t)off[lo] == p;
    }
};

// Longest added token matching at p (which holds the opener byte) that does
// not cross a record start; -1 if none.  AddedVocabulary uses leftmost-longest
// matching; added tokens never overlap because the opener byte occurs only at
// their start (checked on the host).
__device__ int special_match(const DevTok &T, const Src &S, int64_t p) {
    int best = -1, best_len = 0;
    for (int k = 0; k < T.n_special; ++k) {
        int l = T.special_len[k];
        if (p + l > S.N || l <= best_len) continue;
        bool ok = true;
        for (int j = 1; j < l && ok; ++j) ok = S.byte(p + j) == T.special_bytes[k][j] && !S.rstart(p + j);
        if (ok) { best = k; best_len = l; }
    }
    return best;
}

// End of the record containing p (first record start > p), bounded by N.
__device__ int64_t rec_end_of(const Src &S, const int32_t *rb, int nrb, int64_t rb_next, bool rb_ok, int64_t p) {
    if (rb_ok) {
        int rel = (int)(p - S.w0);
        int lo = 0, hi = nrb;
        while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (rb[mid] <= rel) lo = mid + 1; else hi = mid;
        }
        return lo < nrb ? S.w0 + rb[lo] : rb_next;
    }
    int64_t lo = 0, hi = S.R;  // first off[r] > p
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if ((int64_t)S.off[mid] <= p) lo = mid + 1; else hi = mid;
    }
    int64_t e = (int64_t)S.off[lo];
    return e < S.N ? e : S.N;
}

// Unicode table entry of code point cp.
__device__ __forceinline__ uint32_t uentry(const DevTok &T, uint32_t cp) {
    if (cp >= 0x110000u) return UC_DEL;
    return T.uentry[(uint32_t)T.upage[cp >> 7] * 128u + (cp & 127u)];
}

// Strict UTF-8 decode of the char starting at lead byte p (b = its byte);
// the char must not cross a record start.  Invalid -> U+FFFD (class DEL), 1 byte.
__device__ __forceinline__ uint32_t decode(const Src &S, int64_t p, uint32_t b, int *len) {
    int n;
    uint32_t c;
    if ((b & 0xE0) == 0xC0) { n = 2; c = b & 0x1F; }
    else if ((b & 0xF0) == 0xE0) { n = 3; c = b & 0x0F; }
    else if ((b & 0xF8) == 0xF0) { n = 4; c = b & 0x07; }
    else { *len = 1; return 0xFFFD; }
    if (p + n > S.N) { *len = 1; return 0xFFFD; }
    for (int k = 1; k < n; ++k) {
        uint32_t x = S.byte(p + k);
        if ((x & 0xC0) != 0x80 || S.rstart(p + k)) { *len = 1; return 0xFFFD; }
        c = (c << 6) | (x & 0x3F);
    }
    *len = n;
    return c;
}

// Is byte q covered by an added token that starts before q?
__device__ bool covered(const DevTok &T, const Src &S, int64_t q) {
    for (int d = 1; d < T.max_special_len; ++d) {
        if (S.rstart(q - d + 1)) return false;  // q-d lies in an earlier record
        int64_t x = q - d;
        if (x < 0) return false;
        if (S.byte(x) == T.opener) {
            // the opener occurs only at token starts: this is the only candidate
            int m = special_match(T, S, x);
            return m >= 0 && T.special_len[m] > d;
        }
    }
    return false;
}

// Visible class of the char starting at q.  `maybe_special` = an opener byte
// occurs close enough to matter.
__device__ uint8_t vclass(const DevTok &T, const Src &S, const uint32_t *ascii, int64_t q, bool maybe_special) {
    uint32_t b = S.byte(q);
    if ((b & 0xC0) == 0x80) return V_NONE;
    if (maybe_special) {
        if (covered(T, S, q)) return V_NONE;
        if (b == T.opener && special_match(T, S, q) >= 0) return V_SPEC;
    }
    uint32_t e;
    if (b < 0x80) {
        e = ascii[b];
    } else {
        int len;
        uint32_t cp = decode(S, q, b, &len);
        e = uentry(T, cp);
    }
    switch (e & 3u) {
        case UC_OTHER: return V_OTHER;
        case UC_WS: return V_WS;
        case UC_ISO: return V_ISO;
        default: return V_NONE;
    }
}

// ---- WordPiece --------------------------------------------------------------

// Probe the vocab for the literal piece (cont ? "##" : "") + w[start, end).
template <class W>
__device__ int vocab_find(const DevTok &T, const W &w, int start, int end, bool cont) {
    uint64_t h = cont ? T.h_cont : FNV_BASIS;
    for (int i = start; i < end; ++i) h = (h ^ w(i)) * FNV_PRIME;
    const uint32_t len = (uint32_t)(end - start) + (cont ? 2u : 0u);
    const uint32_t tag = (uint32_t)(h >> 32);
    uint32_t s = (uint32_t)h & T.slot_mask;
    for (;;) {
        const uint4 *p = reinterpret_cast<const uint4 *>(T.slots + s);
        uint4 a = p[0];
        if ((int32_t)a.y < 0) return -1;
        if (a.x == tag && a.z == len) {
            uint4 in = p[1];
            uint32_t words[4] = {in.x, in.y, in.z, in.w};
            bool ok = true;
            const int pre = cont ? 2 : 0;
            for (uint32_t k = 0; k < len && ok; ++k) {
                uint32_t q = (int)k < pre ? (uint32_t)'#' : w(start + (int)k - pre);
                uint32_t e;
                if (k < 16) e = (words[k >> 2] >> ((k & 3) * 8)) & 0xFF;
                else e = T.vpool[a.w + k];
                ok = q == e;
            }
            if (ok) return (int)a.y;
        }
        s = (s + 1) & T.slot_mask;
    }
}

// WordPiece::tokenize on the normalized word w[0, L) (byte-addressed, UTF-8),
// writing ids to out[]; returns the id count.  Candidates longer than the
// longest vocabulary piece are skipped: they cannot match, so the greedy
// longest-match result is unchanged.
template <class W>
__device__ int wordpiece(const DevTok &T, const W &w, int L, uint32_t *out) {
    int n = 0, start = 0;
    while (start < L) {
        int lim = start == 0 ? T.maxlen_first : T.maxlen_cont;
        int end = start + lim < L ? start + lim : L;
        while (end < L && end > start && (w(end) & 0xC0) == 0x80) --end;  // char boundary
        int id = -1;
        while (end > start) {
            id = vocab_find(T, w, start, end, start > 0);
            if (id >= 0) break;
            do { --end; } while (end > start && (w(end) & 0xC0) == 0x80);
        }
        if (id < 0) {
            out[0] = (uint32_t)T.unk_id;
            return 1;
        }
        out[n++] = (uint32_t)id;
        start = end;
    }
    return n;
}

struct LdsLower {  // ASCII fast path: word bytes straight from LDS, lower-cased
    const uint8_t *p;
    __device__ __forceinline__ uint32_t operator()(int i) const {
        uint32_t b = p[i];
        return (b - 'A' < 26u) ? b + 32 : b;
    }
};
struct BufBytes {
    const uint8_t *p;
    __device__ __forceinline__ uint32_t operator()(int i) const { return p[i]; }
};

// Appends the normalized bytes of code point cp (table entry e, raw bytes at
// S[p, p+len)) to buf.
__device__ __forceinline__ int append_norm(const DevTok &T, const Src &S, uint32_t e, int64_t p, int len,
                                           uint8_t *buf, int nb) {
    if (e & 4u) {
        for (int k = 0; k < len; ++k) buf[nb + k] = (uint8_t)S.byte(p + k);
        return nb + len;
    }
    const uint8_t *pe = T.upool + (e >> 8);
    int m = pe[0];
    for (int k = 0; k < m; ++k) buf[nb + k] = pe[2 + k];
    return nb + m;
}

// Tokenizes the WORD piece starting at p (an OTHER char after a non-OTHER
// visible char).  The word runs over OTHER and invisible chars until a
// WS/ISO char, an added token or the record end.
__device__ int word_tokens(const DevTok &T, const Src &S, const uint32_t *ascii, int64_t p, int64_t rec_end,
                           uint32_t *out) {
    // pass 1: extent, normalized length, and whether the fast path applies
    int64_t i = p;
    int nchars = 0;
    bool simple = true;  // pure ASCII OTHER chars, all inside the LDS window
    while (i < rec_end) {
        uint32_t b = S.byte(i);
        if (b < 0x80) {
            uint32_t c = ascii[b] & 3u;
            if (c == UC_OTHER) {
                if (T.n_special && b == T.opener && special_match(T, S, i) >= 0) break;
                ++nchars; ++i;
                if (nchars > MAX_WORD_CHARS) break;
                continue;
            }
            if (c == UC_DEL) { simple = false; ++i; continue; }
            break;  // WS or ISO
        }
        simple = false;
        if ((b & 0xC0) == 0x80) { ++i; continue; }  // continuation / stray byte
        int len;
        uint32_t cp = decode(S, i, b, &len);
        uint32_t e = uentry(T, cp);
        uint32_t c = e & 3u;
        if (c == UC_OTHER) {
            nchars += (e & 4u) ? 1 : T.upool[(e >> 8) + 1];
        } else if (c != UC_DEL) {
            break;
        }
        i += len;
        if (nchars > MAX_WORD_CHARS) break;
    }
    if (nchars > MAX_WORD_CHARS) {
        out[0] = (uint32_t)T.unk_id;
        return 1;
    }
    if (simple && S.in_win(p) && S.in_win(i - 1)) {
        LdsLower w{S.win + (p - S.w0)};
        return wordpiece(T, w, (int)(i - p), out);
    }
    // pass 2 (rare): materialize the normalized word in private memory
    uint8_t buf[MAX_WORD_BYTES];
    int nb = 0;
    for (int64_t q = p; q < i;) {
        uint32_t b = S.byte(q);
        if (b < 0x80) {
            uint32_t e = ascii[b];
            if ((e & 3u) == UC_OTHER) buf[nb++] = (uint8_t)((b - 'A' < 26u) ? b + 32 : b);
            ++q;
            continue;
        }
        if ((b & 0xC0) == 0x80) { ++q; continue; }
        int len;
        uint32_t cp = decode(S, q, b, &len);
        uint32_t e = uentry(T, cp);
        if ((e & 3u) == UC_OTHER) nb = append_norm(T, S, e, q, len, buf, nb);
        q += len;
    }
    BufBytes w{buf};
    return wordpiece(T, w, nb, out);
}

// Tokenizes an ISO piece: one isolated char (punctuation or CJK).
__device__ int iso_tokens(const DevTok &T, const Src &S, const uint32_t *ascii, int64_t p, uint32_t *out) {
    uint8_t buf[16];
    int nb;
    uint32_t b = S.byte(p);
    if (b < 0x80) {
        uint32_t e = ascii[b];
        nb = append_norm(T, S, e, p, 1, buf, 0);
    } else {
        int len;
        uint32_t cp = decode(S, p, b, &len);
        nb = append_norm(T, S, uentry(T, cp), p, len, buf, 0);
    }
    BufBytes w{buf};
    return wordpiece(T, w, nb, out);
}

}  // namespace

// -----------------------------------------------------------------------------
__global__ __launch_bounds__(TOK_THREADS) void k_wordpiece_chunks(
    DevTok T, const uint8_t *__restrict__ text, int64_t N, const uint64_t *__restrict__ off, int64_t R,
    uint32_t *__restrict__ tokc, uint32_t *__restrict__ chunk_cnt, uint32_t *__restrict__ rec_local) {
    __shared__ __attribute__((aligned(16))) uint8_t win[WIN];
    __shared__ uint8_t rflag[WIN];
    __shared__ uint8_t vcl[CHUNK];          // visible class per owned byte; later: tokens per piece
    __shared__ uint32_t pieces[CHUNK];      // (pos - c0) | kind << 16
    __shared__ uint32_t stage[STAGE];       // tokens, indexed by piece byte position
    __shared__ uint16_t poff[CHUNK];        // token offset of each piece within the chunk
    __shared__ uint32_t ascii[128];
    __shared__ int32_t rb[RB_CAP];          // record starts inside the window (relative)
    __shared__ uint32_t scratch[TOK_THREADS / 64 + 1];
    __shared__ int64_t sh_misc[4];          // rb_next, r_lo, r_hi, state-in
    __shared__ int sh_nrb;

    const int tid = threadIdx.x;
    const int64_t c0 = (int64_t)blockIdx.x * CHUNK;
    const int64_t c1 = c0 + CHUNK < N ? c0 + CHUNK : N;
    const int64_t w0 = c0 - HALO_L;

    // ---- 1. stage the window; ASCII table ----------------------------------
    for (int v = tid; v < WIN / 16; v += TOK_THREADS) {
        int64_t p = w0 + (int64_t)v * 16;
        uint4 x;
        if (p >= 0 && p + 16 <= N) {
            x = *reinterpret_cast<const uint4 *>(text + p);
        } else {
            uint8_t tmp[16];
            for (int k = 0; k < 16; ++k) tmp[k] = (p + k >= 0 && p + k < N) ? text[p + k] : 0;
            x = *reinterpret_cast<uint4 *>(tmp);
        }
        *reinterpret_cast<uint4 *>(win + v * 16) = x;
        *reinterpret_cast<uint4 *>(rflag + v * 16) = make_uint4(0, 0, 0, 0);
    }
    if (tid < 128) ascii[tid] = T.uentry[(uint32_t)T.upage[0] * 128u + tid];
    if (tid == 0) {
        // records whose start lies in [w0, w0 + WIN]: r in [ra, rb_)
        int64_t lo = 0, hi = R + 1;
        while (lo < hi) { int64_t m = (lo + hi) >> 1; if ((int64_t)off[m] < w0) lo = m + 1; else hi = m; }
        int64_t ra = lo;
        lo = ra; hi = R + 1;
        while (lo < hi) { int64_t m = (lo + hi) >> 1; if ((int64_t)off[m] < w0 + WIN) lo = m + 1; else hi = m; }
        int64_t rz = lo;
        sh_misc[0] = rz <= R ? (int64_t)off[rz] : N;   // next record start after the window
        if (sh_misc[0] > N) sh_misc[0] = N;
        sh_misc[1] = ra;
        sh_misc[2] = rz;
        // owned boundaries: off[r] in [c0, c1)
        lo = 0; hi = R + 1;
        while (lo < hi) { int64_t m = (lo + hi) >> 1; if ((int64_t)off[m] < c0) lo = m + 1; else hi = m; }
        sh_misc[3] = lo;
        sh_nrb = (int)(rz - ra);
    }
    __syncthreads();
    const int64_t rb_next = sh_misc[0];
    const int64_t ra = sh_misc[1];
    const int nrb_all = sh_nrb;
    const bool rb_ok = nrb_all <= RB_CAP;
    for (int k = tid; k < nrb_all; k += TOK_THREADS) {
        int rel = (int)((int64_t)off[ra + k] - w0);
        rflag[rel] = 1;
        if (rb_ok) rb[k] = rel;
    }
    __syncthreads();
    // rb[] is sorted; empty records repeat a start, which the "first start
    // > p" search in rec_end_of tolerates.

    Src S{win, rflag, w0, text, N, off, R};

    // ---- 2. classify owned bytes; per-thread summary of the visible state --
    const int64_t s0 = c0 + (int64_t)tid * BYTES_PER_THREAD;
    const int64_t s1 = s0 + BYTES_PER_THREAD < c1 ? s0 + BYTES_PER_THREAD : c1;
    bool maybe_special = false;
    if (T.n_special) {
        for (int64_t q = s0 - T.max_special_len; q < s1; ++q)
            if (q >= 0 && q < N && S.byte(q) == T.opener) { maybe_special = true; break; }
    }
    // summary encoding: 0 = pass-through, 0x100 | v = state after segment
    uint32_t summ = 0;
    for (int64_t q = s0; q < s1; ++q) {
        if (rflag[q - w0]) summ = 0x100 | V_NONE;
        uint8_t v = vclass(T, S, ascii, q, maybe_special);
        vcl[q - c0] = v;
        if (v != V_NONE) summ = 0x100 | v;
    }

    // state before the chunk: last visible char of the same record before c0
    if (tid == 0) {
        uint32_t st = V_NONE;
        int64_t q = c0 - 1;
        bool msp = T.n_special != 0;
        while (q >= 0 && !S.rstart(q + 1)) {
            int64_t cs = q;
            int k = 0;
            while (k < 3 && cs > 0 && (S.byte(cs) & 0xC0) == 0x80 && !S.rstart(cs)) { --cs; ++k; }
            uint8_t v = vclass(T, S, ascii, cs, msp);
            if (v != V_NONE) {
                // a lead byte whose sequence is invalid does not cover q: its
                // continuation bytes are invisible and the lead itself is DEL,
                // so a visible result always belongs to a char covering q.
                st = v;
                break;
            }
            q = cs - 1;
        }
        scratch[TOK_THREADS / 64] = st;
    }
    __syncthreads();
    const uint32_t chunk_state = scratch[TOK_THREADS / 64];
    const int64_t r_lo = sh_misc[3];
    __syncthreads();

    uint32_t st_in = block_excl_last_scan<TOK_THREADS>(summ, scratch);
    uint32_t state = (st_in & 0x100) ? (st_in & 0xFF) : chunk_state;

    // ---- 3/4. piece starts, block-compacted into pieces[] ---------------------
    uint32_t npt = 0;
    {
        uint32_t sst = state;
        for (int64_t q = s0; q < s1; ++q) {
            if (rflag[q - w0]) sst = V_NONE;
            uint8_t v = vcl[q - c0];
            if (v == V_NONE) continue;
            if (v == V_SPEC || v == V_ISO || (v == V_OTHER && sst != V_OTHER)) ++npt;
            sst = v;
        }
    }
    uint32_t np_total;
    uint32_t pbase = block_excl_sum<TOK_THREADS>(npt, &np_total, scratch);
    {
        uint32_t sst = state;
        for (int64_t q = s0; q < s1; ++q) {
            if (rflag[q - w0]) sst = V_NONE;
            uint8_t v = vcl[q - c0];
            if (v == V_NONE) continue;
            if (v == V_SPEC || v == V_ISO || (v == V_OTHER && sst != V_OTHER))
                pieces[pbase++] = (uint32_t)(q - c0) | ((uint32_t)v << 16);
            sst = v;
        }
    }
    __syncthreads();
    const int np = (int)np_total;

    // ---- 5. tokenize pieces -------------------------------------------------
    uint8_t *cnt = vcl;  // reuse: tokens per piece (<= 100)
    for (int i = tid; i < np; i += TOK_THREADS) {
        uint32_t pc = pieces[i];
        int64_t p = c0 + (pc & 0xFFFF);
        uint32_t kind = pc >> 16;
        uint32_t *out = stage + (pc & 0xFFFF);
        int k;
        if (kind == V_SPEC) {
            int m = special_match(T, S, p);
            out[0] = (uint32_t)T.special_id[m < 0 ? 0 : m];
            k = 1;
        } else if (kind == V_ISO) {
            k = iso_tokens(T, S, ascii, p, out);
        } else {
            int64_t rend = rec_end_of(S, rb, nrb_all, rb_next, rb_ok, p);
            k = word_tokens(T, S, ascii, p, rend, out);
        }
        cnt[i] = (uint8_t)k;
    }
    __syncthreads();

    // ---- 6. compact staged tokens into this chunk's tokc region --------------
    const int per = (np + TOK_THREADS - 1) / TOK_THREADS;
    const int a = tid * per < np ? tid * per : np;
    const int b = a + per < np ? a + per : np;
    uint32_t mine = 0;
    for (int i = a; i < b; ++i) mine += cnt[i];
    uint32_t total;
    uint32_t base = block_excl_sum<TOK_THREADS>(mine, &total, scratch);
    uint32_t *dst = tokc + (int64_t)blockIdx.x * STAGE;
    for (int i = a; i < b; ++i) {
        poff[i] = (uint16_t)base;
        const uint32_t *src = stage + (pieces[i] & 0xFFFF);
        for (int k = 0; k < cnt[i]; ++k) dst[base + k] = src[k];
        base += cnt[i];
    }
    __syncthreads();
    if (tid == 0) chunk_cnt[blockIdx.x] = total;

    // record boundaries owned by this chunk: local token offset of the first
    // piece at or after the boundary
    for (int64_t r = r_lo + tid; r <= R; r += TOK_THREADS) {
        int64_t pos = (int64_t)off[r];
        if (pos >= c1) break;
        int rel = (int)(pos - c0);
        int lo = 0, hi = np;
        while (lo < hi) {
            int m = (lo + hi) >> 1;
            if ((int)(pieces[m] & 0xFFFF) < rel) lo = m + 1; else hi = m;
        }
        rec_local[r] = lo < np ? (uint32_t)poff[lo] : total;
    }
}

hipError_t launch_wordpiece_chunks(const DevTok &T, const uint8_t *text, int64_t N, const uint64_t *off, int64_t R,
                                   uint32_t *tokc, uint32_t *chunk_cnt, uint32_t *rec_local, hipStream_t st) {
    const int64_t n_chunks = (N + CHUNK - 1) / CHUNK;
    if (n_chunks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_wordpiece_chunks, dim3((unsigned)n_chunks), dim3(TOK_THREADS), 0, st, T, text, N, off, R,
                       tokc, chunk_cnt, rec_local);
    return hipGetLastError();
}

}  // namespace sdl
