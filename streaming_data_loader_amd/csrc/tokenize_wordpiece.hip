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
// assembly (pipeline.hip).
//
// One wave64 workgroup owns CHUNK = 1024 bytes of the arena; lane t owns
// bytes [c0 + 16t, c0 + 16t + 16):
//   1. each lane loads its 16 bytes with one 16-B non-temporal load (they stay
//      in VGPRs) and stores them into an LDS window [c0-32, c0+1024+32);
//      record starts in the window become an LDS bitmap;
//   2. classification is register-resident: an arithmetic ASCII classifier
//      packs 16 four-bit visible classes into one u64; only lead bytes >= 0xC0
//      (two-level Unicode table in L2) and added-token openers take a loop;
//   3. a wave scan carries the last visible class across lanes; piece starts
//      (words, isolated chars, added tokens) are compacted into an LDS list;
//   4. each lane WordPiece-tokenizes pieces i, i+64, ...: an ASCII word of
//      <= 16 bytes is read from LDS as 5 aligned dwords + v_alignbyte,
//      lower-cased and classified with SWAR, and every candidate piece is one
//      hash of 4 dwords + one 32-B probe of the L2-resident vocab table whose
//      slots hold the piece bytes inline; other words take a general path;
//   5. staged ids (LDS, indexed by piece byte position: a piece never has
//      more ids than bytes) are compacted into this chunk's slice of `tokc`,
//      and each record boundary's local id offset is recorded.
#include "common.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "tok_device.hpp"

#include <cstdio>

namespace sdl {

namespace {

// ASCII visible class (same as the table's ASCII rows; checked on the host)
__device__ __forceinline__ uint32_t ascii_vclass(uint32_t b) {
    const uint32_t l = b | 0x20u;
    if (l - 'a' < 26u || b - '0' < 10u) return V_OTHER;
    if (b == ' ' || b == '\t' || b == '\n' || b == '\r') return V_WS;
    if (b < 32u || b == 127u) return V_NONE;
    return V_ISO;
}

// ascii_vclass of 4 bytes as 4 nibbles (bytes >= 0x80: V_NONE)
__device__ __forceinline__ uint32_t vclass4(uint32_t x) {
    const uint32_t lo7 = ~x & B7, a = x & 0x7F7F7F7Fu;
    const uint32_t an = swar_alnum(x);
    const uint32_t ws = (in7(a, 9, 10) | in7(a, 13, 13) | in7(a, ' ', ' ')) & lo7;
    const uint32_t ctl = ~ge7(a, 32) | ge7(a, 127);  // includes \t \n \r (ws wins)
    const uint32_t iso = lo7 & ~an & ~ws & ~ctl;
    return nibpack4(((an | ws) >> 7) | ((an | iso) >> 6));  // OTHER 3, WS 1, ISO 2, NONE 0
}

// Device Unicode entry (assets.cpp: device_entry): bits 0-1 class, bit 2
// identity, bit 3 inline (bits 4-5 nbytes-1, 6-7 nchars-1, 8-31 the bytes),
// else bits 8-31 = pool offset.  One load for the BMP, two beyond it.
__device__ __forceinline__ uint32_t uentry(const DevTok &T, uint32_t cp) {
    if (cp < 0x10000u) return T.ubmp[cp].x;
    if (cp >= 0x110000u) return UC_DEL;
    return T.uentry[(uint32_t)T.upage[cp >> 7] * 128u + (cp & 127u)];
}
__device__ __forceinline__ int entry_nchars(const DevTok &T, uint32_t e) {
    if (e & 4u) return 1;
    if (e & 8u) return (int)((e >> 6) & 3u) + 1;
    return T.upool[(e >> 8) + 1];
}

__device__ __forceinline__ uint32_t vclass_of_entry(uint32_t e) {
    switch (e & 3u) {
        case UC_OTHER: return V_OTHER;
        case UC_WS: return V_WS;
        case UC_ISO: return V_ISO;
        default: return V_NONE;
    }
}

// Full visible class of the char at q (general path).
__device__ __forceinline__ uint32_t vclass_general(const Ctx &C, int64_t q) {
    const DevTok &T = *C.T;
    const uint32_t b = C.byte(q);
    if ((b & 0xC0u) == 0x80u) return V_NONE;
    if (T.n_special) {
        for (int d = 1; d < T.max_special_len; ++d) {  // covered by an earlier added token?
            if (C.rstart(q - d + 1)) break;
            const int64_t x = q - d;
            if (x < 0) break;
            if (C.byte(x) == T.opener) {
                const int m = special_match(C, x);
                if (m >= 0 && T.special_len[m] > d) return V_NONE;
                break;
            }
        }
        if (b == T.opener && special_match(C, q) >= 0) return V_SPEC;
    }
    if (b < 0x80u) return ascii_vclass(b);
    int len;
    return vclass_of_entry(uentry(T, decode(C, q, b, &len)));
}

// ---- WordPiece ------------------------------------------------------------------

// WordPiece::tokenize over a normalized word held in a byte buffer.
__device__ __forceinline__ int wordpiece_general(const DevTok &T, const uint8_t *w, int L, lds_u16 *out) {
    int n = 0, start = 0;
    while (start < L) {
        const int lim = start == 0 ? T.maxlen_first : T.maxlen_cont;
        int end = start + lim < L ? start + lim : L;
        while (end < L && end > start && (w[end] & 0xC0) == 0x80) --end;
        int id = -1;
        while (end > start) {
            id = probe_general(T, w, start, end, start > 0 ? 1u : 0u);
            if (id >= 0) break;
            do { --end; } while (end > start && (w[end] & 0xC0) == 0x80);
        }
        if (id < 0) {
            out[0] = (uint16_t)T.unk_id;
            return 1;
        }
        out[n++] = (uint16_t)id;
        start = end;
    }
    return n;
}

// Appends the normalized bytes of a non-ASCII OTHER/ISO char.
template <typename Buf>
__device__ __forceinline__ int append_norm(const Ctx &C, uint32_t e, int64_t p, int len, Buf *buf, int nb) {
    if (e & 4u) {
        for (int k = 0; k < len; ++k) buf[nb + k] = (uint8_t)C.byte(p + k);
        return nb + len;
    }
    if (e & 8u) {
        const int m = (int)((e >> 4) & 3u) + 1;
        for (int k = 0; k < m; ++k) buf[nb + k] = (uint8_t)(e >> (8 + 8 * k));
        return nb + m;
    }
    const uint8_t *pe = C.T->upool + (e >> 8);
    const int m = pe[0];
    for (int k = 0; k < m; ++k) buf[nb + k] = pe[2 + k];
    return nb + m;
}

__device__ __forceinline__ int utf8_len(uint32_t lead) {
    return lead < 0x80u ? 1 : (lead & 0xE0u) == 0xC0u ? 2 : (lead & 0xF0u) == 0xE0u ? 3 : 4;
}

// Extent of the general WORD piece at p: it runs over OTHER and invisible
// chars until a WS/ISO char, an added token or the record end.  Counts its
// normalized chars (stops past MAX_WORD_CHARS) and bytes.
__device__ __forceinline__ int64_t word_extent(const Ctx &C, int64_t p, int64_t rec_end, int *nchars_out, int *nbytes_out) {
    const DevTok &T = *C.T;
    int64_t i = p;
    int nchars = 0, nbytes = 0;
    while (i < rec_end && nchars <= MAX_WORD_CHARS) {
        const uint32_t b = C.byte(i);
        if (b < 0x80u) {
            const uint32_t c = ascii_vclass(b);
            if (c == V_OTHER) {
                if (T.n_special && b == T.opener && special_match(C, i) >= 0) break;
                ++nchars;
                ++nbytes;
                ++i;
                continue;
            }
            if (c == V_NONE) { ++i; continue; }
            break;
        }
        if ((b & 0xC0u) == 0x80u) { ++i; continue; }
        int len;
        const uint32_t e = uentry(T, decode(C, i, b, &len));
        const uint32_t c = e & 3u;
        if (c == UC_OTHER) {
            nchars += entry_nchars(T, e);
            nbytes += (e & 4u) ? len : (e & 8u) ? (int)((e >> 4) & 3u) + 1 : (int)T.upool[e >> 8];
        } else if (c != UC_DEL) {
            break;
        }
        i += len;
    }
    *nchars_out = nchars;
    *nbytes_out = nbytes;
    return i;
}

// Normalized bytes of the word [p, i) into buf (private or LDS); returns the
// count.  NFD canonical ordering of the kept combining marks: a run of them is
// appended as it comes and sorted in place (stable, by ccc) when a starter --
// kept, removed or inside a precomposed char -- ends it.
template <typename Buf>
__device__ __forceinline__ int word_materialize(const Ctx &C, int64_t p, int64_t i, Buf *buf) {
    const DevTok &T = *C.T;
    int nb = 0;
    int run = -1;
    auto ccc_at = [&](int x, int l) {
        uint32_t cp = l == 2 ? buf[x] & 0x1Fu : l == 3 ? buf[x] & 0x0Fu : buf[x] & 0x07u;
        for (int k = 1; k < l; ++k) cp = (cp << 6) | (buf[x + k] & 0x3Fu);
        return (uentry(T, cp) >> 8) & 0xFFu;
    };
    auto flush = [&]() {
        if (run < 0) return;
        for (bool swapped = true; swapped;) {
            swapped = false;
            for (int x = run; x < nb;) {
                const int l1 = utf8_len(buf[x]);
                if (x + l1 >= nb) break;
                const int l2 = utf8_len(buf[x + l1]);
                if (ccc_at(x, l1) > ccc_at(x + l1, l2)) {
                    uint8_t t[4];
                    for (int k = 0; k < l1; ++k) t[k] = buf[x + k];
                    for (int k = 0; k < l2; ++k) buf[x + k] = buf[x + l1 + k];
                    for (int k = 0; k < l1; ++k) buf[x + l2 + k] = t[k];
                    swapped = true;
                    x += l2;
                } else {
                    x += l1;
                }
            }
        }
        run = -1;
    };
    auto push = [&](uint32_t bytes, int l) {
        if (run < 0) run = nb;
        for (int k = 0; k < l; ++k) buf[nb++] = (uint8_t)(bytes >> (8 * k));
    };
    for (int64_t q = p; q < i;) {
        const uint32_t b = C.byte(q);
        if (b < 0x80u) {
            if (ascii_vclass(b) == V_OTHER) {
                flush();
                buf[nb++] = (uint8_t)((b - 'A' < 26u) ? b + 32u : b);
            }
            ++q;
            continue;
        }
        if ((b & 0xC0u) == 0x80u) { ++q; continue; }
        int len;
        const uint32_t e = uentry(T, decode(C, q, b, &len));
        const uint32_t cls = e & 3u;
        if ((e & 24u) == 16u) {  // canonical ordering entry
            if (cls == UC_DEL) {
                flush();  // a removed starter ends the run
            } else if (e & 4u) {  // a kept mark
                uint32_t bytes = 0;
                for (int k = 0; k < len; ++k) bytes |= C.byte(q + k) << (8 * k);
                push(bytes, len);
            } else {  // precomposed: its starters end the run, its kept marks join it
                const uint8_t *pe = T.upool + (e >> 8);
                const int m = pe[0];
                for (int x = 0; x < m;) {
                    const uint32_t lead = pe[2 + x];
                    const int l = utf8_len(lead);
                    uint32_t cp = l == 1 ? lead : l == 2 ? lead & 0x1Fu : l == 3 ? lead & 0x0Fu : lead & 0x07u;
                    uint32_t bytes = lead;
                    for (int k = 1; k < l; ++k) {
                        cp = (cp << 6) | (pe[2 + x + k] & 0x3Fu);
                        bytes |= (uint32_t)pe[2 + x + k] << (8 * k);
                    }
                    const uint32_t e2 = uentry(T, cp);
                    if ((e2 & 24u) == 16u && (e2 & 4u) && (e2 & 3u) == UC_OTHER) {
                        push(bytes, l);
                    } else {
                        flush();
                        for (int k = 0; k < l; ++k) buf[nb++] = (uint8_t)(bytes >> (8 * k));
                    }
                    x += l;
                }
            }
        } else if (cls == UC_OTHER) {
            flush();
            nb = append_norm(C, e, q, len, buf, nb);
        }
        q += len;
    }
    flush();
    return nb;
}

// General WORD piece materialized in private memory, WordPiece one probe at a
// time (words whose normalization exceeds the LDS lattice buffer).
__device__ __forceinline__ int word_general(const Ctx &C, int64_t p, int64_t rec_end, lds_u16 *out) {
    int nchars, nbytes;
    const int64_t i = word_extent(C, p, rec_end, &nchars, &nbytes);
    if (nchars > MAX_WORD_CHARS) {
        out[0] = (uint16_t)C.T->unk_id;
        return 1;
    }
    uint8_t buf[MAX_WORD_BYTES];
    const int nb = word_materialize(C, p, i, buf);
    return wordpiece_general(*C.T, buf, nb, out);
}

// Bytes [off, off + 16) of an LDS byte buffer (dword aligned, readable 20
// bytes past off) in registers, the first n kept.
__device__ __forceinline__ W16 lds_w16(const lds_u32 *b32, int off, int n) {
    const int a = off >> 2;
    const uint32_t sh = (uint32_t)(off & 3);
    const uint32_t x0 = b32[a], x1 = b32[a + 1], x2 = b32[a + 2], x3 = b32[a + 3], x4 = b32[a + 4];
    return keep_bytes(W16{__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh),
                          __builtin_amdgcn_alignbyte(x3, x2, sh), __builtin_amdgcn_alignbyte(x4, x3, sh)},
                      n < 16 ? n : 16);
}

// start of the char that ends right before byte `end` (UTF-8 in registers)
__device__ __forceinline__ int w16_prev_char(const W16 &w, int end, int start) {
    int e = end - 1;
    while (e > start && (w16_byte(w, e) & 0xC0u) == 0x80u) --e;
    return e;
}

// BertNormalizer output of the WORD piece at p (or of the single ISO char at
// p if iso) into registers.  Returns false if the normalized word does not fit
// in 16 bytes (then the scratch path handles it, including the 100-char rule).
__device__ __forceinline__ bool normalize_w16(const Ctx &C, int64_t p, int64_t rec_end, bool iso, W16 &w, int &L) {
    const DevTok &T = *C.T;
    w = W16{0, 0, 0, 0};
    int nb = 0;
    int64_t i = p;
    while (i < rec_end) {
        const uint32_t b = C.byte(i);
        if (b < 0x80u) {
            const uint32_t c = ascii_vclass(b);
            if (iso || c == V_OTHER) {
                if (!iso && T.n_special && b == T.opener && special_match(C, i) >= 0) break;
                if (nb >= 16) return false;
                w16_put(w, nb++, (b - 'A' < 26u) ? b + 32u : b);
                ++i;
                if (iso) break;
                continue;
            }
            if (c == V_NONE) { ++i; continue; }
            break;
        }
        if ((b & 0xC0u) == 0x80u) { ++i; continue; }
        int len;
        const uint32_t e = uentry(T, decode(C, i, b, &len));
        const uint32_t c = e & 3u;
        if (c == UC_OTHER && (e & 24u) == 16u) return false;  // canonical ordering: the general path
        if (iso || c == UC_OTHER) {
            if (e & 4u) {
                if (nb + len > 16) return false;
                for (int k = 0; k < len; ++k) w16_put(w, nb++, C.byte(i + k));
            } else if (e & 8u) {
                const int m = (int)((e >> 4) & 3u) + 1;
                if (nb + m > 16) return false;
                for (int k = 0; k < m; ++k) w16_put(w, nb++, (e >> (8 + 8 * k)) & 0xFFu);
            } else {
                const uint8_t *pe = T.upool + (e >> 8);
                const int m = pe[0];
                if (nb + m > 16) return false;
                for (int k = 0; k < m; ++k) w16_put(w, nb++, pe[2 + k]);
            }
            i += len;
            if (iso) break;
            continue;
        }
        if (c == UC_DEL) { i += len; continue; }
        break;
    }
    L = nb;
    return true;
}

// Record end (first record start > p, p in the window) for the general paths:
// the next bit of the window's record-start bitmap, else the first start past
// the window (rb_next).
__device__ __forceinline__ int64_t rec_end_of(const Ctx &C, int64_t rb_next, int64_t p) {
    const int b = (int)(p - C.w0) + 1;
    for (int wd = b >> 5; wd < RBITS_WORDS; ++wd) {
        uint32_t m = C.rbits[wd];
        if (wd == (b >> 5)) m &= ~0u << (b & 31);
        if (m) return C.w0 + 32 * wd + __builtin_ctz(m);
    }
    return rb_next;
}

}  // namespace

// Diagnostic build (-DSDL_STAMPS): wave 0 of every block adds the s_memtime
// cycles spent between phase boundaries (each right after a barrier) into
// sdl_phase_cycles[]; the host prints them.  Never compiled into the product.
#ifdef SDL_STAMPS
__device__ unsigned long long sdl_phase_cycles[16];
#define PHASE_STAMP(k)                                                                  \
    do {                                                                              \
        if (threadIdx.x == 0) {                                                       \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();              \
            atomicAdd(&sdl_phase_cycles[k], t_ - stamp_prev_);                        \
            stamp_prev_ = t_;                                                         \
        }                                                                             \
    } while (0)
#else
#define PHASE_STAMP(k) \
    do {             \
    } while (0)
#endif

// Waves per SIMD the register budget is cut to: 5 (96 VGPRs).  6 (80 VGPRs)
// was 1% faster before the deferred-word lattice; with it, 80 VGPRs spill and
// 5 measures faster on both corpora (fixture 1.868 -> 1.818 ms, held-out
// 2.98 -> 2.86 ms).  LDS (7.1 KB per one-wave block) admits ~5.5 anyway; one
// more 64-B array (7.7 KB) cost 7%.
constexpr int WP_WAVES = 5;
// candidate lengths the pending-word state machine probes per step (longest
// first).  3 and 4 were measured: parity-green and no faster (4: 96 VGPRs,
// fixture 1.14 -> 1.19 ms, held-out 2.32 -> 2.40; 3: within noise) -- the
// machine is bound by its lanes' probe latency, not by its step count.
constexpr int WP_NPROBE = 2;
__global__ __launch_bounds__(TOK_THREADS) __attribute__((amdgpu_waves_per_eu(WP_WAVES, 8))) void k_wordpiece_chunks(
    DevTok T, const uint8_t *__restrict__ text, int64_t N, const uint64_t *__restrict__ off, int64_t R,
    const uint32_t *__restrict__ ranges, uint32_t *__restrict__ tokc, uint32_t *__restrict__ chunk_cnt,
    uint32_t *__restrict__ rec_local, int64_t c_begin) {
    __shared__ __attribute__((aligned(16))) uint8_t s_win[WIN];
    __shared__ uint32_t s_rbits[RBITS_WORDS + 1];
    __shared__ uint16_t s_pieces[CHUNK];   // (pos - c0) | kind << 12
    __shared__ uint16_t s_stage[STAGE];    // ids staged at their piece's byte position
    __shared__ uint8_t s_cnt[CHUNK];       // ids per piece
    __shared__ uint16_t s_pend[PEND_CAP];  // pending piece indices (step 4b)
    __shared__ uint32_t s_scratch[TOK_THREADS / 64 + 3];
    // non-ASCII chars found by the rare pass: [0, 32) a WS/ISO char starts at the
    // chunk position (a word before it ends there), [32, 64) an ISO char whose id
    // is already in its stage slot
    __shared__ uint32_t s_nabits[2 * CHUNK / 32];

    const int tid = threadIdx.x;
#ifdef SDL_STAMPS
    unsigned long long stamp_prev_ = __builtin_amdgcn_s_memtime();
#endif
    const int64_t ci = c_begin + xcd_chunk();  // this block's chunk
    const int64_t c0 = ci * CHUNK;
    const int64_t c1 = c0 + CHUNK < N ? c0 + CHUNK : N;
    const int64_t w0 = c0 - HALO_L;
    const lds_u8 *win = (const lds_u8 *)s_win;
    const lds_u32 *rbits = (const lds_u32 *)s_rbits;

    // ---- 1. load -------------------------------------------------------------
    const uint4 v = load16(text, c0 + 16 * tid, N);
    uint4 hv = make_uint4(0u, 0u, 0u, 0u);
    int64_t hp = 0;
    if (tid < (WIN - CHUNK) / 16) {  // left and right halo pieces
        hp = tid < HALO_L / 16 ? w0 + 16 * tid : c0 + CHUNK + 16 * (tid - HALO_L / 16);
        hv = load16(text, hp, N);
    }
    const int64_t ra = ranges[3 * ci], rz = ranges[3 * ci + 1], r_lo = ranges[3 * ci + 2];
    *reinterpret_cast<uint4 *>(s_win + HALO_L + 16 * tid) = v;
    if (tid < (WIN - CHUNK) / 16) *reinterpret_cast<uint4 *>(s_win + (hp - w0)) = hv;
    if (tid <= RBITS_WORDS) s_rbits[tid] = 0;
    s_nabits[tid] = 0u;  // 2 * CHUNK / 32 == TOK_THREADS words
    const int nrb = (int)(rz - ra);
    int64_t rb_next = rz <= R ? (int64_t)off[rz] : N;
    if (rb_next > N) rb_next = N;
    __syncthreads();
    for (int k = tid; k < nrb; k += TOK_THREADS) {
        const int rel = (int)((int64_t)off[ra + k] - w0);
        atomicOr(&s_rbits[rel >> 5], 1u << (rel & 31));
    }
    __syncthreads();
    PHASE_STAMP(1);

    const Ctx C{&T, win, rbits, w0, text, N, off, R};
#ifdef SDL_ABLATE
    // diagnostic build (tools/build_variants.py abl3=SDL_ABLATE, tools/pmc_calibration.py): load only; every record gets 0 ids (so later stages stay in bounds)
    {  // (an opaque use of the window keeps its loads: `x & 0u` let the compiler drop them all)
        const uint32_t x = s_win[HALO_L + (ci & 1023)];
        asm volatile("" ::"v"(x));
    }
    if (tid == 0) chunk_cnt[ci] = 0u;
    for (int64_t r = r_lo + tid; r <= R && (int64_t)off[r] < c1; r += TOK_THREADS) rec_local[r] = 0;
    return;
#endif

    // ---- 2. register-resident classification of the lane's 16 bytes ----------
    const int64_t s0 = c0 + 16 * tid;
    const int nown = s0 >= c1 ? 0 : (int)(c1 - s0 < 16 ? c1 - s0 : 16);
    const int rel0 = HALO_L + 16 * tid;  // window index of s0 (multiple of 16)
    const uint32_t rmask = (rbits[rel0 >> 5] >> (rel0 & 31)) & 0xFFFFu;
    const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
    uint64_t cls = 0;
    uint32_t leads = 0, opens = 0;
    const uint32_t o4 = T.opener * 0x01010101u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t x = wv[j];
        cls |= (uint64_t)vclass4(x) << (16 * j);
        leads |= gather4(x & (x << 1)) << (4 * j);  // >= 0xC0
        opens |= gather4(~nzb(x ^ o4)) << (4 * j);
    }
    if (!T.n_special) opens = 0;
    if (nown < 16) {
        cls &= nown ? ((1ull << (4 * nown)) - 1ull) : 0ull;
        leads &= (1u << nown) - 1u;
        opens &= (1u << nown) - 1u;
    }
    uint8_t *s_ovr = s_cnt;
    *reinterpret_cast<uint4 *>(s_ovr + 16 * tid) = make_uint4(~0u, ~0u, ~0u, ~0u);
    // Rare bytes are classified block-parallel, one per thread, and returned as
    // per-byte class overrides in LDS (s_cnt doubles as the override array and
    // s_pieces as the work list until the pieces are found):
    //   (a) non-ASCII lead bytes: decode + two-level Unicode table;
    //   (b) added tokens: every opener byte that starts a match marks its bytes
    //       (SPEC at the start, invisible after); applied after (a).
    // tid 0 also owns openers in [c0 - max_special_len + 1, c0): a token starting
    // there may cover this chunk's first bytes
    uint32_t opens_left = 0;
    if (T.n_special && tid == 0) {
        for (int d = 1; d < T.max_special_len; ++d)
            if (c0 - d >= 0 && C.byte(c0 - d) == T.opener) opens_left |= 1u << (d - 1);
    }
    uint32_t nrare;
    const uint32_t rare_n = (uint32_t)__builtin_popcount(leads) |
                            ((uint32_t)(__builtin_popcount(opens) + __builtin_popcount(opens_left)) << 16);
    const uint32_t rbase = block_excl_sum<TOK_THREADS>(rare_n, &nrare, s_scratch);
    const uint32_t n_leads = nrare & 0xFFFFu, n_opens = nrare >> 16;
    {
        uint32_t lb = rbase & 0xFFFFu, ob = n_leads + (rbase >> 16);
        for (uint32_t m = leads; m;) {
            const int i = __builtin_ctz(m);
            m &= m - 1;
            s_pieces[lb++] = (uint16_t)(HALO_L + 16 * tid + i);
        }
        for (uint32_t m = opens; m;) {
            const int i = __builtin_ctz(m);
            m &= m - 1;
            s_pieces[ob++] = (uint16_t)(HALO_L + 16 * tid + i);
        }
        for (uint32_t m = opens_left; m;) {
            const int d = __builtin_ctz(m) + 1;
            m &= m - 1;
            s_pieces[ob++] = (uint16_t)(HALO_L - d);
        }
    }
    __syncthreads();
    PHASE_STAMP(2);
    for (uint32_t k = tid; k < n_leads; k += TOK_THREADS) {
        const int wi = s_pieces[k];
        const int rel = wi - HALO_L;
        int len;
        const uint32_t cp = decode(C, w0 + wi, win[wi], &len);
        // (a canonical BMP char: its entry and its precomputed one-char id in one load)
        const uint2 ue = (len == 2 && cp >= 0x80u) || (len == 3 && cp >= 0x800u) ? T.ubmp[cp]
                                                                                 : make_uint2(uentry(T, cp), 0u);
        const uint32_t e = ue.x;
        const uint32_t vc = vclass_of_entry(e);
        s_ovr[rel] = (uint8_t)vc;
        if (vc == V_WS || vc == V_ISO) atomicOr(&s_nabits[rel >> 5], 1u << (rel & 31));
        // an ISO char is a piece of its own: when it normalizes to one char of <= 16
        // bytes, its WordPiece is one probe of that char (no "##" piece can start
        // inside a char), done here so the piece skips the pending pass
        if (ue.y >> 31) {
            s_stage[rel] = (uint16_t)ue.y;
            atomicOr(&s_nabits[CHUNK / 32 + (rel >> 5)], 1u << (rel & 31));
        } else if (vc == V_ISO && (e & 24u) != 16u && ((e & 4u) || ((e & 8u) && ((e >> 6) & 3u) == 0u))) {
            W16 w{0, 0, 0, 0};
            int L;
            if (e & 4u) {
                L = len;
                for (int q = 0; q < len; ++q) w16_put(w, q, win[wi + q]);
            } else {
                L = (int)((e >> 4) & 3u) + 1;
                for (int q = 0; q < L; ++q) w16_put(w, q, (e >> (8 + 8 * q)) & 0xFFu);
            }
            const int id = L <= T.maxlen_first ? probe_result(probe_load(T, hash16(w, (uint32_t)L, 0u)), (uint32_t)L, w)
                                               : -1;
            s_stage[rel] = (uint16_t)(id >= 0 ? id : T.unk_id);
            atomicOr(&s_nabits[CHUNK / 32 + (rel >> 5)], 1u << (rel & 31));
        }
    }
    PHASE_STAMP(12);
    if (n_opens) {  // block-uniform
        __syncthreads();
        for (uint32_t k = n_leads + tid; k < n_leads + n_opens; k += TOK_THREADS) {
            const int wi = s_pieces[k];
            const int64_t x = w0 + wi;
            const int m = special_match(C, x);
            if (m < 0) continue;
            const int l = T.special_len[m];
            for (int j = 0; j < l; ++j) {
                const int64_t y = x + j;
                if (y >= c0 && y < c1) s_ovr[y - c0] = (uint8_t)(j == 0 ? V_SPEC : V_NONE);
            }
        }
    }
    __syncthreads();
    PHASE_STAMP(3);
    {
        const uint4 o = *reinterpret_cast<const uint4 *>(s_ovr + 16 * tid);
        const uint32_t ov[4] = {o.x, o.y, o.z, o.w};
        uint64_t onib = 0, keep = 0;  // override classes, nibbles without one (0xFF)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            onib |= (uint64_t)nibpack4(ov[j] & 0x0F0F0F0Fu) << (16 * j);
            keep |= (uint64_t)nibpack4(fullb(ov[j] & B7) & 0x0F0F0F0Fu) << (16 * j);
        }
        cls = (cls & keep) | (onib & ~keep);
    }
    // Each byte's previous visible class, byte-parallel: a record start at byte
    // i + 1 puts a stopper (8) at byte i, then the visible classes and stoppers
    // fill forward over the invisible bytes in four doubling steps.
    constexpr uint64_t NIB1 = 0x1111111111111111ull;
    auto nib_zero = [](uint64_t x) -> uint64_t {  // 1 at the base bit of every zero nibble
        return ~(x | (x >> 1) | (x >> 2) | (x >> 3)) & NIB1;
    };
    const uint64_t stop = nib_spread(rmask >> 1);
    uint64_t fill = (cls & ~((stop << 4) - stop)) | (stop << 3);
#pragma unroll
    for (int sh = 4; sh < 64; sh <<= 1) {
        const uint64_t z = nib_zero(fill);
        fill |= (fill << sh) & ((z << 4) - z);
    }
    // lane summary for the carry scan: 0 = pass-through, 0x100 | v = state after
    const uint32_t last = (uint32_t)(fill >> 60);
    const uint32_t summ = (last != 0u || (rmask & 1u)) ? 0x100u | (last & 7u) : 0u;
    // state before the chunk: last visible char of the same record before c0
    if (tid == 0) {
        uint32_t st = V_NONE;
        int64_t q = c0 - 1;
        while (q >= 0 && !C.rstart(q + 1)) {
            int64_t cs = q;
            int k = 0;
            while (k < 3 && cs > 0 && (C.byte(cs) & 0xC0u) == 0x80u && !C.rstart(cs)) { --cs; ++k; }
            const uint32_t vc = vclass_general(C, cs);
            if (vc != V_NONE) { st = vc; break; }
            q = cs - 1;
        }
        s_scratch[TOK_THREADS / 64] = st;
    }
    __syncthreads();
    const uint32_t chunk_state = s_scratch[TOK_THREADS / 64];
    __syncthreads();
    PHASE_STAMP(4);
    const uint32_t st_in = block_excl_last_scan<TOK_THREADS>(summ, s_scratch);

    // ---- 3. piece starts -------------------------------------------------------
    uint32_t pmask;
    {
        const uint32_t st = (rmask & 1u) ? (uint32_t)V_NONE : (st_in & 0x100u) ? (st_in & 0xFFu) : chunk_state;
        uint64_t pv = fill << 4;  // previous visible class (stopper 8: none)
        const uint64_t z = nib_zero(pv);  // nothing visible before in the lane: the incoming state
        pv = (pv | (((z << 4) - z) & (NIB1 * st))) & 0x7777777777777777ull;
        const uint64_t is_o = nib_zero(cls ^ (NIB1 * V_OTHER));
        const uint64_t is_si = nib_zero(cls ^ (NIB1 * V_ISO)) | nib_zero(cls ^ (NIB1 * V_SPEC));
        uint64_t m = (is_si | (is_o & ~nib_zero(pv ^ (NIB1 * V_OTHER)))) & NIB1;  // bit 4i: a piece starts at byte i
        m = (m | (m >> 3)) & 0x0303030303030303ull;
        m = (m | (m >> 6)) & 0x000F000F000F000Full;
        m = (m | (m >> 12)) & 0x000000FF000000FFull;
        pmask = (uint32_t)((m | (m >> 24)) & 0xFFFFull);
    }
    uint32_t np_total;
    uint32_t pbase = block_excl_sum<TOK_THREADS>((uint32_t)__builtin_popcount(pmask), &np_total, s_scratch);
    for (uint32_t m = pmask; m;) {
        const int i = __builtin_ctz(m);
        m &= m - 1;
        const uint32_t c = (uint32_t)(cls >> (4 * i)) & 0xFu;
        s_pieces[pbase++] = (uint16_t)((16 * tid + i) | (c << 12));
    }
    __syncthreads();
    PHASE_STAMP(5);
    const int np = (int)np_total;

    // ---- 4. tokenize pieces ---------------------------------------------------------
    // (a) every lane sets up TOK_UNROLL pieces at a time and issues their
    //     full-word probes back to back, so most words (in-vocabulary, <= 16 B)
    //     finish with one latency and TOK_UNROLL loads in flight per lane;
    //     added tokens and one-byte punctuation finish without a probe;
    // (b) the rest (misses, collisions, longer or non-ASCII words) go to a
    //     pending list that a per-lane state machine drains: lanes pull work
    //     from a block-wide LDS queue and advance one vocab probe per iteration,
    //     so no lane idles behind a long word.
    // (a) and (b) alternate in rounds so the pending list stays within
    // PEND_CAP (a round of (a) adds at most TOK_THREADS * TOK_UNROLL).
    lds_u16 *stage = (lds_u16 *)s_stage;
    if (tid == 0) {
        s_scratch[TOK_THREADS / 64 + 1] = 0;  // pending count
        s_scratch[TOK_THREADS / 64 + 2] = 0;  // deferred count
    }
    __syncthreads();
    PHASE_STAMP(10);
    const int lane = tid & 63;
    const lds_u32 *w32 = (const lds_u32 *)s_win;
    // word setup shared by (a) and (b): returns false if the general path is needed
    auto word_setup = [&](int prel, W16 &lw, int &Lout) -> bool {
        const int wr = prel + HALO_L;
        const int a = wr >> 2;
        const uint32_t sh = (uint32_t)(wr & 3);
        const uint32_t x0 = w32[a], x1 = w32[a + 1], x2 = w32[a + 2], x3 = w32[a + 3], x4 = w32[a + 4];
        const W16 raw{__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh),
                      __builtin_amdgcn_alignbyte(x3, x2, sh), __builtin_amdgcn_alignbyte(x4, x3, sh)};
        const uint32_t b16 = (x4 >> (8 * sh)) & 0xFFu;  // byte at p + 16
        const uint32_t om = msb4(swar_alnum(raw.x)) | (msb4(swar_alnum(raw.y)) << 4) |
                            (msb4(swar_alnum(raw.z)) << 8) | (msb4(swar_alnum(raw.w)) << 12);
        int Lw = __builtin_ctz(~om);  // leading ASCII letters/digits, <= 16
        const int rb0 = wr + 1;     // a record start at p+1 .. p+16 ends the word
        const uint64_t rw = ((uint64_t)rbits[(rb0 >> 5) + 1] << 32) | rbits[rb0 >> 5];
        const uint32_t rbm = (uint32_t)(rw >> (rb0 & 31)) & 0xFFFFu;
        const int Lr = rbm ? __builtin_ctz(rbm) + 1 : 17;
        bool fast;
        if (Lr <= Lw) {
            Lw = Lr;
            fast = true;
        } else {
            const uint32_t t =
                Lw < 16 ? (((Lw < 4 ? raw.x : Lw < 8 ? raw.y : Lw < 12 ? raw.z : raw.w) >> (8 * (Lw & 3))) & 0xFFu) : b16;
            const uint32_t tc = vclass4(t) & 0xFu;  // t >= 0x80: V_NONE
            const int te = prel + Lw;  // a non-ASCII WS/ISO char there ends the word too
            const uint32_t na = t >= 0xC0u && te < CHUNK ? (s_nabits[te >> 5] >> (te & 31)) & 1u : 0u;
            fast = (((0x6u >> tc) & 1u) | na) != 0u || c0 + prel + Lw >= N;  // WS, ISO
        }
        lw = keep_bytes(W16{swar_lower(raw.x), swar_lower(raw.y), swar_lower(raw.z), swar_lower(raw.w)}, Lw);
        Lout = Lw;
        return fast;
    };
    for (int r0 = 0; r0 < np;) {
    // (a) batched first probes
    for (; r0 < np && (int)s_scratch[TOK_THREADS / 64 + 1] <= PEND_CAP - TOK_THREADS * TOK_UNROLL;
         r0 += TOK_THREADS * TOK_UNROLL) {
        uint32_t hsh[TOK_UNROLL], key[TOK_UNROLL];
        W16 cand[TOK_UNROLL];
        int prel_u[TOK_UNROLL], L_u[TOK_UNROLL];
        bool probe[TOK_UNROLL], pend[TOK_UNROLL];
#pragma unroll
        for (int u = 0; u < TOK_UNROLL; ++u) {
            const int pi = r0 + u * TOK_THREADS + tid;
            probe[u] = pend[u] = false;
            hsh[u] = key[u] = 0;
            L_u[u] = 0;
            cand[u] = W16{0, 0, 0, 0};
            prel_u[u] = 0;
            if (pi >= np) continue;
            const uint32_t pc = s_pieces[pi];
            const int prel = (int)(pc & 0xFFFu);
            const uint32_t kind = pc >> 12;
            prel_u[u] = prel;
            if (kind == V_SPEC) {
                const int m = special_match(C, c0 + prel);
                stage[prel] = (uint16_t)T.special_id[m < 0 ? 0 : m];
                s_cnt[pi] = 1;
            } else if (kind == V_ISO) {
                const uint32_t b = win[prel + HALO_L];
                if (b < 0x80u) {
                    stage[prel] = (uint16_t)T.ascii_id[b];
                    s_cnt[pi] = 1;
                } else if ((s_nabits[CHUNK / 32 + (prel >> 5)] >> (prel & 31)) & 1u) {
                    s_cnt[pi] = 1;  // its id is in its stage slot (rare pass)
                } else {
                    pend[u] = true;
                }
            } else {
                W16 lw;
                int Lw;
                if (word_setup(prel, lw, Lw) && Lw <= T.maxlen_first) {
                    cand[u] = lw;
                    L_u[u] = Lw;
                    key[u] = (uint32_t)Lw;
                    hsh[u] = hash16(lw, (uint32_t)Lw, 0u);
                    probe[u] = true;
                } else {
                    pend[u] = true;
                }
            }
        }
        Probe pr[TOK_UNROLL];
#pragma unroll
        for (int u = 0; u < TOK_UNROLL; ++u) pr[u] = probe_load(T, hsh[u]);
#pragma unroll
        for (int u = 0; u < TOK_UNROLL; ++u) {
            const int pi = r0 + u * TOK_THREADS + tid;
            if (probe[u]) {
                const int id = probe_result(pr[u], key[u], cand[u]);
                if (id >= 0) {
                    stage[prel_u[u]] = (uint16_t)id;
                    s_cnt[pi] = 1;
                } else {
                    pend[u] = true;
                }
            }
            const uint64_t pm = __ballot(pend[u]);
            if (pm) {
                const int leader = __builtin_ctzll(pm);
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(&s_scratch[TOK_THREADS / 64 + 1], (uint32_t)__popcll(pm));
                base = lane_bcast(base, leader);
                if (pend[u]) s_pend[base + __popcll(pm & ((1ull << lane) - 1ull))] = (uint16_t)pi;
            }
        }
        __syncthreads();  // the pending count is read by the loop test
    }
    PHASE_STAMP(11);
    int npend = (int)s_scratch[TOK_THREADS / 64 + 1];
    if (tid == 0) s_scratch[TOK_THREADS / 64 + 1] = 0;  // becomes the queue head
    __syncthreads();
    // (b) state machine over the pending pieces.  A pending word is worked by a group of G
    //     lanes (G = 64 / pending lanes, at most 8; wave-uniform): the group's lanes hold the same
    //     word state, lane g probes the candidates g * WP_NPROBE .. (g + 1) * WP_NPROBE - 1
    //     chars shorter than the longest remaining one, and the group takes the longest hit --
    //     the lowest lane with one -- so a step covers G * WP_NPROBE candidate lengths of
    //     WordPiece's longest-match-first walk instead of WP_NPROBE (a chunk holds ~12 pending
    //     words on held-out text, ~1 on the fixture: most lanes would otherwise idle).
    if (npend) {
        const int G = npend <= 8 ? 8 : npend > 32 ? 1 : 64 / npend;  // (lanes past the last group idle)
        const int gl = lane % G, g0 = lane - gl;    // lane in the group, the group's first lane
        const uint64_t gmask = ((1ull << G) - 1ull) << g0;
        const bool grouped = g0 + G <= 64;
        bool exhausted = !grouped;  // (a lane outside every group takes no word)
        bool active = false;  // a fast WordPiece state is live (the same in every lane of a group)
        int pi = 0, prel = 0, L = 0, start = 0, end = 0, nout = 0;
        W16 w{0, 0, 0, 0};
        for (;;) {
            const bool need = !active && !exhausted;
            const uint64_t nm = __ballot(need && gl == 0);
            if (nm) {
                const int leader = __builtin_ctzll(nm);
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(&s_scratch[TOK_THREADS / 64 + 1], (uint32_t)__popcll(nm));
                base = lane_bcast(base, leader);
                int q = (int)base + __popcll(nm & ((1ull << lane) - 1ull));  // (valid in the group's first lane)
                if (G > 1) q = __shfl(q, g0);
                if (need) {
                    if (q >= npend) {
                        exhausted = true;
                    } else {
                        pi = s_pend[q];
                        const uint32_t pc = s_pieces[pi];
                        prel = (int)(pc & 0xFFFu);
                        const uint32_t kind = pc >> 12;
                        const int64_t p = c0 + prel;
                        lds_u16 *out = stage + prel;
                        bool fits;
                        if (kind == V_OTHER && word_setup(prel, w, L)) {
                            fits = true;
                        } else {
                            fits = normalize_w16(C, p, rec_end_of(C, rb_next, p),
                                                 kind == V_ISO, w, L);
                        }
                        if (fits) {
                            start = 0;
                            end = L < T.maxlen_first ? L : T.maxlen_first;
                            while (end < L && end > 0 && (w16_byte(w, end) & 0xC0u) == 0x80u) --end;
                            nout = 0;
                            active = end > 0;
                            if (!active && gl == 0) {  // no piece can match: the word is [UNK]
                                out[0] = (uint16_t)T.unk_id;
                                s_cnt[pi] = 1;
                            }
                        } else if (gl == 0) {
                            if (kind == V_ISO) {
                                int len;
                                const uint32_t e = uentry(T, decode(C, p, win[prel + HALO_L], &len));
                                uint8_t buf[16];
                                const int nb = append_norm(C, e, p, len, buf, 0);
                                s_cnt[pi] = (uint8_t)wordpiece_general(T, buf, nb, out);
                            } else {  // deferred to the cooperative lattice below
                                const uint32_t d = atomicAdd(&s_scratch[TOK_THREADS / 64 + 2], 1u);
                                s_pend[d] = (uint16_t)pi;  // d < this round's consumed entries
                            }
                        }
                    }
                }
            }
            if (!__any(active || !exhausted)) break;
            if (active) {  // probe this lane's WP_NPROBE candidates, gl * WP_NPROBE chars below `end`
                const W16 sh = start ? shift_right_bytes(w, start) : w;
                const uint32_t cont = start > 0 ? 1u : 0u;
                int ek[WP_NPROBE];
                // (an ASCII word's chars are its bytes: no walk over continuation bytes)
                const bool ascii = ((w.x | w.y | w.z | w.w) & 0x80808080u) == 0u;
                int e0 = end;
                if (ascii) {
                    e0 = end - gl * WP_NPROBE > start ? end - gl * WP_NPROBE : start;
                } else {
                    for (int k = 0; k < gl * WP_NPROBE; ++k) e0 = e0 > start ? w16_prev_char(w, e0, start) : start;
                }
                ek[0] = e0;
#pragma unroll
                for (int k = 1; k < WP_NPROBE; ++k)
                    ek[k] = ek[k - 1] <= start ? start : ascii ? ek[k - 1] - 1 : w16_prev_char(w, ek[k - 1], start);
                W16 cw[WP_NPROBE];
                Probe Pk[WP_NPROBE];
#pragma unroll
                for (int k = 0; k < WP_NPROBE; ++k) {
                    const int nk = ek[k] - start;
                    cw[k] = keep_bytes(sh, nk);
                    Pk[k] = probe_load(T, hash16(cw[k], (uint32_t)nk, cont));
                }
                int id = -1, got = 0;
#pragma unroll
                for (int k = 0; k < WP_NPROBE; ++k) {
                    const int nk = ek[k] - start;
                    if (id < 0 && nk > 0) {
                        id = probe_result(Pk[k], (uint32_t)nk | (cont << 8), cw[k]);
                        got = nk;
                    }
                }
                int e1 = ek[WP_NPROBE - 1];
                if (G > 1) {  // the group's longest hit: its lowest lane with one
                    const uint64_t hm = __ballot(id >= 0) & gmask;
                    const int src = hm ? __builtin_ctzll(hm) : g0;
                    id = __shfl(id, src);
                    got = __shfl(got, src);
                    e1 = __shfl(e1, g0 + G - 1);
                }
                const int n1 = e1 - start;
                lds_u16 *out = stage + prel;
                if (id >= 0) {
                    if (gl == 0) out[nout] = (uint16_t)id;
                    ++nout;
                    start += got;
                    if (start >= L) {
                        if (gl == 0) s_cnt[pi] = (uint8_t)nout;
                        active = false;
                    } else {
                        end = L < start + T.maxlen_cont ? L : start + T.maxlen_cont;
                        while (end < L && end > start && (w16_byte(w, end) & 0xC0u) == 0x80u) --end;
                    }
                } else {
                    end = n1 > 0 ? w16_prev_char(w, e1, start) : start;
                    if (end <= start) {  // no piece matches here: the whole word is [UNK]
                        if (gl == 0) {
                            out[0] = (uint16_t)T.unk_id;
                            s_cnt[pi] = 1;
                        }
                        active = false;
                    }
                }
            }
        }
        // (c) deferred words (normalization longer than 16 bytes, DEL runs,
        //     canonical ordering): one at a time, normalized by lane 0 into LDS
        //     (the pending list's space, free now), then the WordPiece lattice:
        //     every (start, length) candidate with a vocab piece of that length
        //     is one probe task dealt across the wave, and each start keeps its
        //     longest hit (atomic max of length << 16 | id); lane 0 walks
        //     greedy longest-match-first over them.  Probe latencies per word
        //     ~ candidates / 64, where probing one candidate at a time pays one
        //     per candidate.
        __syncthreads();
        const int ndef = (int)s_scratch[TOK_THREADS / 64 + 2];
        if (ndef) {
            uint32_t dl[PEND_CAP / 64];
#pragma unroll
            for (int j = 0; j < PEND_CAP / 64; ++j) {
                const int d = 64 * j + lane;
                dl[j] = d < ndef ? s_pend[d] : 0u;
            }
            __syncthreads();
            lds_u8 *wb = (lds_u8 *)s_pend;
            const lds_u32 *wb32 = (const lds_u32 *)s_pend;
            lds_u32 *best = (lds_u32 *)s_pend + LW_BUF / 4;
            for (int d = 0; d < ndef; ++d) {
                uint32_t mine = dl[0];
#pragma unroll
                for (int j = 1; j < PEND_CAP / 64; ++j)
                    if ((d >> 6) == j) mine = dl[j];
                const int dpi = lane_bcast((int)mine, d & 63);
                const int dprel = (int)(s_pieces[dpi] & 0xFFFu);
                const int64_t dp = c0 + dprel;
                lds_u16 *dout = stage + dprel;
                int dL = 0;
                if (lane == 0) {
                    const int64_t rend = rec_end_of(C, rb_next, dp);
                    int nch, nby;
                    const int64_t iend = word_extent(C, dp, rend, &nch, &nby);
                    if (nch > MAX_WORD_CHARS) {
                        dout[0] = (uint16_t)T.unk_id;
                        s_cnt[dpi] = 1;
                    } else if (nby > LW_MAX || T.wp_long_pieces) {
                        s_cnt[dpi] = (uint8_t)word_general(C, dp, rend, dout);
                    } else {
                        dL = word_materialize(C, dp, iend, wb);
                        for (int k = dL; k < dL + 20; ++k) wb[k] = 0;
                    }
                }
                dL = lane_bcast(dL, 0);
                if (dL == 0) continue;  // wave-uniform
                for (int k = lane; k < dL; k += 64) best[k] = 0u;
                __syncthreads();
                const int nf = T.wp_nlens[0], nc = T.wp_nlens[1];
                const int ntask = nf + (dL - 1) * nc;
                for (int k = lane; k < ntask; k += 64) {
                    int st, n;
                    if (k < nf) {
                        st = 0;
                        n = T.wp_lens[k];
                    } else {
                        st = 1 + (k - nf) / nc;
                        n = T.wp_lens[LW_MAX + (k - nf) % nc];
                    }
                    if (st + n > dL || (wb[st] & 0xC0u) == 0x80u || (st + n < dL && (wb[st + n] & 0xC0u) == 0x80u))
                        continue;
                    const uint32_t cont = st > 0 ? 1u : 0u;
                    uint32_t h = hinit((uint32_t)n, cont);
                    for (int b0 = 0; b0 < n; b0 += 16) {
                        const W16 blk = lds_w16(wb32, st + b0, n - b0);
                        h = hmix(hmix(hmix(hmix(h, blk.x), blk.y), blk.z), blk.w);
                    }
                    h = hfinal(h);
                    const W16 first = lds_w16(wb32, st, n);
                    const Probe P = probe_load(T, h);
                    const uint32_t key = (uint32_t)n | (cont << 8);
                    int id = -1;
                    for (int which = 0; which < 2 && id < 0; ++which) {
                        const uint4 a = which ? P.a2 : P.a1, b = which ? P.b2 : P.b1;
                        if (!slot_match(a, b, key, first)) continue;
                        bool ok = true;
                        for (int x = 16; x < n && ok; ++x) ok = T.vpool[a.z + x] == wb[st + x];
                        if (ok) id = (int32_t)a.y;
                    }
                    if (id >= 0)
                        __hip_atomic_fetch_max(best + st, ((uint32_t)n << 16) | (uint32_t)id, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                __syncthreads();
                if (lane == 0) {
                    int nout = 0;
                    for (int st = 0; st < dL;) {
                        const uint32_t bv = best[st];
                        if (!bv) {
                            nout = -1;
                            break;
                        }
                        dout[nout++] = (uint16_t)(bv & 0xFFFFu);
                        st += (int)(bv >> 16);
                    }
                    if (nout < 0) {
                        dout[0] = (uint16_t)T.unk_id;
                        nout = 1;
                    }
                    s_cnt[dpi] = (uint8_t)nout;
                }
                __syncthreads();
            }
        }
    }
    __syncthreads();
    if (tid == 0) {
        s_scratch[TOK_THREADS / 64 + 1] = 0;  // the next round's pending count
        s_scratch[TOK_THREADS / 64 + 2] = 0;  // ... and deferred count
    }
    __syncthreads();
    }
    PHASE_STAMP(7);

    // ---- 5. compact ids into this chunk's tokc slice ------------------------------
    const int per = (np + TOK_THREADS - 1) / TOK_THREADS;
    const int a0 = tid * per < np ? tid * per : np;
    const int a1 = a0 + per < np ? a0 + per : np;
    uint32_t mine = 0;
    for (int i = a0; i < a1; ++i) mine += s_cnt[i];
    uint32_t total;
    const uint32_t base0 = block_excl_sum<TOK_THREADS>(mine, &total, s_scratch);
    uint32_t *dst = tokc + ci * STAGE;
    uint32_t base = base0;
    // non-temporal stores: the lists are read once, by the compaction, and must
    // not evict the vocabulary table from L2 (rows 0.39 -> 0.34 ms measured).
    // The list is first packed in LDS (the text window is dead now) so the wave
    // writes it as whole 16-B lanes: scattered 4-B non-temporal stores cost
    // 3.5x the list's bytes in HBM writes (PMC WRITE_SIZE 851 MB vs 240 MB).
    if (total <= (uint32_t)(WIN / 2)) {
        lds_u16 *packed = (lds_u16 *)s_win;
        for (int i = a0; i < a1; ++i) {
            const int prel = s_pieces[i] & 0xFFF;
            const int k = s_cnt[i];
            for (int j = 0; j < k; ++j) packed[base + j] = s_stage[prel + j];
            base += k;
        }
        __syncthreads();
        const lds_u32 *p32 = (const lds_u32 *)s_win;
        for (uint32_t e = 4u * (uint32_t)tid; e < total; e += 4u * TOK_THREADS) {
            const uint32_t x = p32[e >> 1], y = p32[(e >> 1) + 1];
            u32x4 v;
            v.x = x & 0xFFFFu;
            v.y = x >> 16;
            v.z = y & 0xFFFFu;
            v.w = y >> 16;
            __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(dst + e));
        }
    } else {
        for (int i = a0; i < a1; ++i) {
            const int prel = s_pieces[i] & 0xFFF;
            const int k = s_cnt[i];
            for (int j = 0; j < k; ++j) __builtin_nontemporal_store((uint32_t)s_stage[prel + j], dst + base + j);
            base += k;
        }
    }
    __syncthreads();
    // the stage is free now: it holds each piece's id offset in the chunk
    uint16_t *s_poff = s_stage;
    base = base0;
    for (int i = a0; i < a1; ++i) {
        s_poff[i] = (uint16_t)base;
        base += s_cnt[i];
    }
    __syncthreads();
    PHASE_STAMP(8);
    if (tid == 0) chunk_cnt[ci] = total;
    // record boundaries owned by this chunk: local id offset of the first piece
    // at or after the boundary
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
    PHASE_STAMP(9);
}

#ifdef SDL_STAMPS
void print_phase_cycles() {
    unsigned long long h[16];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(sdl_phase_cycles), sizeof(h)) != hipSuccess) return;
    static const char *names[] = {"", "load+rbits", "classify+lists", "rare-openers+sync", "merge+lookback",
                                  "scan+pieces", "-", "wp-pending", "compact", "rec_local", "wp-init",
                                  "wp-first-probes", "rare-leads"};
    unsigned long long tot = 0;
    for (int k = 1; k <= 12; ++k) tot += h[k];
    fprintf(stderr, "[stamps] block-cycles by phase (wave 0, all blocks, all calls):");
    for (int k = 1; k <= 12; ++k)
        if (k != 6) fprintf(stderr, " %s=%.1f%%", names[k], 100.0 * h[k] / (tot ? tot : 1));
    fprintf(stderr, " total=%llu\n", tot);
}
#endif

hipError_t launch_wordpiece_chunks(const DevTok &T, const uint8_t *text, int64_t N, const uint64_t *off, int64_t R,
                                   uint32_t *ranges, uint32_t *tokc, uint32_t *chunk_cnt, uint32_t *rec_local,
                                   hipStream_t st, int64_t c_begin, int64_t c_end) {
    const int64_t n_chunks = (N + CHUNK - 1) / CHUNK;
    if (c_end < 0 || c_end > n_chunks) c_end = n_chunks;
    if (c_begin < 0) c_begin = 0;
    if (c_end <= c_begin) return hipSuccess;
    hipLaunchKernelGGL(k_wordpiece_chunks, dim3((unsigned)(c_end - c_begin)), dim3(TOK_THREADS), 0, st, T, text, N,
                       off, R, ranges, tokc, chunk_cnt, rec_local, c_begin);
    return hipGetLastError();
}

}  // namespace sdl
