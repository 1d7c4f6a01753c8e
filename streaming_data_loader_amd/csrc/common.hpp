// common.hpp -- definitions shared by the host library and the gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

namespace sdl {

// ---- Unicode table classes (tools/make_unicode_tables.py) -----------------
enum : uint32_t { UC_OTHER = 0, UC_WS = 1, UC_ISO = 2, UC_DEL = 3 };

// ---- visible class of a char start, as BertPreTokenizer sees it ------------
// NONE = invisible (continuation byte, DEL char, byte covered by an added token)
enum : uint8_t { V_NONE = 0, V_WS = 1, V_ISO = 2, V_OTHER = 3, V_SPEC = 4 };

// ---- tokenize workgroup geometry -----------------------------------------
constexpr int TOK_THREADS = 64;                   // one wave64 per workgroup: no cross-wave stalls
constexpr int CHUNK = 1024;                       // text bytes owned by one workgroup (16 per lane)
constexpr int BYTES_PER_THREAD = CHUNK / TOK_THREADS;
constexpr int HALO_L = 32;                        // look-back bytes staged in LDS
constexpr int HALO_R = 32;                        // look-ahead bytes staged in LDS
constexpr int WIN = HALO_L + CHUNK + HALO_R;      // 1088 bytes of text in LDS
constexpr int STAGE = CHUNK + 128;                // token slots per chunk (>= tokens owned)
constexpr int TOK_UNROLL = 2;        // first probes in flight per lane (2: no spills at 5 waves/SIMD)
constexpr int PEND_CAP = 256;            // WordPiece pieces pending the state machine (LDS)
constexpr int RB_CAP = 256;                       // record starts listed in LDS per window
constexpr int MAX_WORD_CHARS = 100;               // WordPiece max_input_chars_per_word
constexpr int MAX_WORD_BYTES = 4 * MAX_WORD_CHARS + 8;
constexpr int RAND_MAX_S = 2048;  // rng_mode 1: longest row the shuffle kernel holds in LDS
constexpr int LW_MAX = 96;   // WordPiece: longest normalized word for the LDS lattice (bytes)
constexpr int LW_BUF = 128;  // ... its byte buffer (LW_MAX + 20 readable), then u32 best[LW_MAX]

constexpr int MAX_SPECIAL = 8;
constexpr int MAX_SPECIAL_LEN = 24;
constexpr int MAX_FRAME = 4;


// Vocabulary cuckoo hash table: every piece sits in one of its two slots, so
// any lookup (hit or miss) is one round trip of two independent 32-B reads.
// A piece is keyed by (payload, cont), cont = it starts with "##" and payload
// is the rest.  Slot: w0 key = payload length | cont << 8, w1 id (-1 = empty),
// w2 offset of the payload in the pool, w3 the piece hash (host only),
// w4..w7 the first 16 payload bytes (zero padded).
struct alignas(32) VSlot {
    uint32_t key;
    int32_t id;
    uint32_t pool_off;
    uint32_t hash;
    uint8_t inl[16];
};

// piece hash: init(len, cont); per zero-padded 16-byte block, 4 little-endian
// dwords mixed in; final avalanche (assets.cpp: piece_hash runs the same steps).
__host__ __device__ inline uint32_t ph_init(uint32_t len, uint32_t cont) {
    return (len * 2u + cont) * 0x9E3779B1u ^ 0x7F4A7C15u;
}
__host__ __device__ inline uint32_t ph_mix(uint32_t h, uint32_t w) {
    h ^= w;
    h *= 0x85EBCA6Bu;
    return h ^ (h >> 13);
}
__host__ __device__ inline uint32_t ph_final(uint32_t h) {
    h ^= h >> 16;
    h *= 0x7FEB352Du;
    h ^= h >> 15;
    h *= 0x846CA68Bu;
    return h ^ (h >> 16);
}
// the two cuckoo slots of a piece hash
__host__ __device__ inline uint32_t cuckoo_slot1(uint32_t h, uint32_t mask) { return h & mask; }
__host__ __device__ inline uint32_t cuckoo_slot2(uint32_t h, uint32_t mask) {
    uint32_t g = (h >> 16) | (h << 16);
    g *= 0xD35A2D97u;
    g ^= g >> 15;
    return g & mask;
}
static_assert(sizeof(VSlot) == 32, "VSlot must be 32 bytes");
static_assert(PEND_CAP % 64 == 0 && 2 * PEND_CAP >= LW_BUF + 4 * LW_MAX, "the WordPiece lattice buffer reuses the pending list");

// Byte-level BPE merge table (cuckoo, 2 slots of 8 B): key = left id << 16 |
// right id, val = rank << 16 | merged id; empty slot key = 0xFFFFFFFF.
struct MSlot {
    uint32_t key;
    uint32_t val;
};
__host__ __device__ inline uint32_t merge_hash(uint32_t key) { return ph_final(key * 0x9E3779B1u + 0x632BE5ABu); }
constexpr uint32_t MERGE_NONE = 0xFFFFu;  // rank of a pair with no merge

// GPT-2 regex classes of a code point (tools/make_gpt2_tables.py)
enum : uint32_t { GC_O = 0, GC_L = 1, GC_N = 2, GC_W = 3 };

enum : int32_t { TOK_WORDPIECE = 0, TOK_BYTE_BPE = 1, TOK_UNIGRAM = 2 };

// ---- Unigram (t5) ------------------------------------------------------------
// Vocab slot key cont values: 0 piece without "▁", 1 piece "▁"+payload,
// 2 word-table entry (payload = an ASCII word, id field = packed Viterbi
// result of "▁"+word: (k << 24) | x, x = the id when k == 1, else the offset
// of its k ids in DevTok.wres), 3 added token (payload = its raw bytes).
enum : uint32_t { UC_PIECE = 0, UC_META = 1, UC_WORD = 2, UC_ADDED = 3 };
constexpr int UNI_STAGE = 2 * CHUNK + 128; // tokc entries per chunk (a 1-byte word can yield 2 ids)
constexpr int UNI_WMAX = 16;        // longest word (bytes) the chunk kernel settles itself
constexpr int UNI_NODES = UNI_WMAX + 4;
// A chunk's tokc slice (UNI_STAGE u32): its entry list (<= STAGE entries: every piece's ids fit
// the stage slots up to the next piece) and, behind it, the Viterbi jobs the chunk kernel hands
// to k_unigram_viterbi -- a job's ids land as u16 at its stage position in the results region,
// and its list entry becomes LMARK | UNI_JOB_BIT | k << 24 (6 bits) | position (k_compact_tokens expands it).
constexpr int UNI_VPC = 88;                           // Viterbi jobs per chunk, and 16-B payload units (more: long items)
constexpr int UNI_VMAX = 48;                          // longest job payload (printable ASCII words past UNI_WMAX)
constexpr int UNI_VRING = 20;                         // the Viterbi DP's node ring: jobs past UNI_WMAX need
                                                      // maxlen_first < UNI_VRING and maxlen_meta + 3 < UNI_VRING
constexpr int UNI_JR_OFF = STAGE;                     // results: u16 [STAGE] at the stage positions
constexpr int UNI_JP_OFF = STAGE + STAGE / 2;         // job payloads: uint4 [UNI_VPC], ceil(L / 16) (>= 1) each
constexpr int UNI_JM_OFF = UNI_JP_OFF + 4 * UNI_VPC;  // job metas: L | pos << 6 | entry << 18
constexpr int UNI_JN_OFF = UNI_JM_OFF + UNI_VPC;      // the chunk's job count
constexpr uint32_t UNI_JOB_BIT = 0x40000000u;
static_assert(UNI_JN_OFF < UNI_STAGE && (UNI_JP_OFF * 4) % 16 == 0 && (UNI_STAGE * 4) % 16 == 0,
              "the Viterbi jobs fit the tokc slice behind its list");
constexpr int UNI_LANE_NORM = 256;  // normalized bytes per lane of the long-item kernel
constexpr int UNI_HUGE_NORM = 1 << 18;  // ... per wave of the huge-item kernel
// grapheme / whitespace properties (tools/make_t5_tables.py)
enum : uint32_t { GB_OTHER = 0, GB_CR, GB_LF, GB_CONTROL, GB_EXTEND, GB_ZWJ, GB_RI, GB_PREPEND, GB_SPACING,
                  GB_L, GB_V, GB_T, GB_LV, GB_LVT };
constexpr uint32_t GP_EXTPICT = 0x10u, GP_WS = 0x80u;
// White_Space (char::is_whitespace; tools/make_t5_tables.py WHITE_SPACE) and the
// property byte of an ASCII char, as arithmetic: the host checks the loaded
// tables agree (sdl_batcher.cpp), so the kernels test them without a load
__host__ __device__ inline bool uni_white_space(uint32_t cp) {
    if (cp < 0x80u) return (cp >= 9u && cp <= 13u) || cp == 32u;
    return cp == 0x85u || cp == 0xA0u || cp == 0x1680u || cp - 0x2000u <= 0xAu || cp == 0x2028u || cp == 0x2029u ||
           cp == 0x202Fu || cp == 0x205Fu || cp == 0x3000u;
}
__host__ __device__ inline uint32_t uni_ascii_props(uint32_t c) {
    const uint32_t gcb = c == 13u ? GB_CR : c == 10u ? GB_LF : (c < 32u || c == 127u) ? GB_CONTROL : GB_OTHER;
    return gcb | (uni_white_space(c) ? GP_WS : 0u);
}
// per-code-point entry of the t5 normalizer (x, y):
//   x bits 0-7 grapheme/whitespace properties, bit 8 the char is a charsmap
//   key, bit 9 it is a proper prefix of a longer key, bit 10 its normalization
//   is inline in y (bits 11-13: byte count 0..4), else y = offset of the
//   NUL-terminated normalization in the charsmap's string blob.
constexpr uint32_t CP_KEY = 1u << 8, CP_PREFIX = 1u << 9, CP_INLINE = 1u << 10;

// Everything a tokenize kernel needs, passed by value as a kernel argument.
struct DevTok {
    int32_t kind;            // TOK_*
    const uint2 *ubmp;       // U+0000..U+FFFF (flat): device Unicode entry, WordPiece one-char ISO id (assets.cpp)
    const uint16_t *upage;   // Unicode page table  [0x110000/128]
    const uint32_t *uentry;  // Unicode blocks      [n_blocks*128]
    const uint8_t *upool;    // normalized strings  (u8 nbytes, u8 nchars, bytes)
    const VSlot *slots;      // vocab hash table
    const uint8_t *vpool;    // vocab piece payload bytes
    const int32_t *ascii_id; // id of each one-byte ASCII word (or [UNK])
    uint32_t slot_mask;
    int32_t unk_id;
    int32_t maxlen_first;    // longest non-"##" piece (bytes)
    int32_t maxlen_cont;     // longest "##" piece without the prefix (bytes)
    int32_t wp_nlens[2];     // WordPiece: distinct payload lengths <= LW_MAX of non-"##" / "##" pieces,
    const uint8_t *wp_lens;  // ... ascending: [0, LW_MAX) non-"##", [LW_MAX, 2 LW_MAX) "##"
    int32_t wp_long_pieces;  // some piece payload is longer than LW_MAX
    int32_t n_special;       // added tokens matched on the raw text
    int32_t max_special_len;
    uint32_t opener;         // first byte shared by every added token
    int32_t special_id[MAX_SPECIAL];
    uint8_t special_len[MAX_SPECIAL];
    uint8_t special_bytes[MAX_SPECIAL][MAX_SPECIAL_LEN];
    // byte-level BPE (kind == TOK_BYTE_BPE); slots/vpool then hold the word
    // table: every vocab string whose own BPE is itself, keyed by its raw bytes
    const uint16_t *gpage;   // code point page (256) -> class block
    const uint8_t *gblock;   // 64-byte blocks of 2-bit GC_* classes
    const MSlot *mslots;     // merge table
    const uint16_t *byte_id; // id of each single byte symbol
    uint32_t mslot_mask;
    // Unigram (kind == TOK_UNIGRAM): slots hold pieces and added tokens, wslots
    // the word table (UC_* cont values, payloads in vpool); specials are
    // matched "<...>" by hash
    const double *uscore;    // score of each id
    const float *uscore32;   // ... nearest f32 (the slots carry it with its f64 correction)
    const uint16_t *wres;    // word-table results with more than one id
    const VSlot *wslots;     // word table (UC_WORD entries; `slots` holds pieces + added tokens)
    uint32_t wslot_mask;
    const uint16_t *cpage;   // per-code-point entry pages (0x110000/256)
    const uint2 *cent;       // entry blocks of 256 (CP_* layout)
    const uint2 *cbmp;       // ... flattened for U+0000..U+FFFF (one load per BMP char)
    const uint32_t *trie;    // Precompiled charsmap: double-array units
    const uint8_t *tnorm;    // ... and its NUL-separated normalized strings
    uint32_t trie_units, tnorm_len;
    double unk_score;        // min score - 10 (models/unigram/model.rs)
    int32_t maxlen_meta;     // longest "▁"-piece payload (bytes)
    int32_t maxlen_word;     // longest word-table payload
    int32_t maxlen_piece;    // longest piece, "▁" included (bytes)
    const uint8_t *upfx;     // longest plain piece (>= 4 B) under each hashed 4-byte prefix (uni_pfx_key)
};

// Unigram prefix bound: a plain piece of >= 4 bytes starting with bytes x (little-endian u32) is
// at most upfx[uni_pfx_key(x)] bytes long (assets.cpp; a collision only raises the bound)
constexpr int UNI_PFX_BITS = 16;
__host__ __device__ inline uint32_t uni_pfx_key(uint32_t x) { return (x * 0x9E3779B1u) >> (32 - UNI_PFX_BITS); }

// Row assembly parameters (GenTokenizer + BertData/GptData/T5Data framing).
struct RowParams {
    int32_t task;            // SDL_TASK_*
    int32_t B, S;
    int32_t chunk;           // GenTokenizer.chunk
    int32_t min_ids;         // gen_batcher.rs:74 filter on framed length
    int32_t mask_length, mask_id;
    int32_t label_width;
    int32_t n_pre, n_post;   // framing ids around the tokenizer output
    int32_t pre[MAX_FRAME];
    int32_t post[MAX_FRAME];
    uint64_t seed;
    uint64_t first_record;
    int32_t rng_mode;              // MLM masks: 0 Philox contract, 1 rand 0.8.5 StdRng (k_mask_rand)
    // rng_mode 1: the rows' mask bits (S/32 words a row, bit p = position p masked).  Rows known
    // before tokenizing -- chunk 0 of every record, chunk 1 of records of >= mask_spec1 bytes
    // (rand_pre_slot) -- are walked beside the tokenizer (k_mask_rand_rec + k_mask_bits_rec) into
    // mask_bits0 (slot r, and R + mask_spos[r] for chunk 1: the record's place in the list of
    // those, k_rand_spec_list; null: none); k_rows' LATE pass walks the others (rand_rows16).
    // mask_off / mask_R: the call's record offsets and count.
    const uint32_t *mask_bits0;
    const uint32_t *mask_spos;
    const uint64_t *mask_off;
    int64_t mask_R, mask_spec1;
    int32_t mask_w;
    // span (T5Data): trunc(avg - z) draws as CDF tables (RNG contract) and
    // the <extra_id_k> ids (device pointer, 100 entries)
    int32_t gap_kmin, gap_n, size_kmin, size_n;
    uint32_t gap_thr[32], size_thr[32];
    const int32_t *extra_ids;
    // span rng_mode 1: the reference's own draws (rand_distr StandardNormal)
    double avg_span_gap, avg_span_size;
    const double *zig_x, *zig_f;   // ZIG_NORM_X / ZIG_NORM_F (257 each, device)
};

__host__ __device__ inline uint32_t ceil_div_u32(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

// f(std::integral_constant<int, i>) for i = A .. B - 1, in order (a compile-time index for DPP controls)
template <int A, int B, class F>
__device__ __forceinline__ void static_for(const F &f) {
    if constexpr (A < B) {
        f(std::integral_constant<int, A>{});
        static_for<A + 1, B>(f);
    }
}

// rng_mode 1: mask_bits0 slot of row (record r, chunk k) when it was walked beside the tokenizer,
// else -1 (no text is read: the record's byte length from its offsets)
__device__ __forceinline__ int64_t rand_pre_slot(const RowParams &P, int64_t r, uint32_t k) {
    if (!P.mask_bits0) return -1;
    if (k == 0) return r;
    if (k == 1 && P.mask_spec1 > 0 && (int64_t)(P.mask_off[r + 1] - P.mask_off[r]) >= P.mask_spec1)
        return P.mask_R + P.mask_spos[r];
    return -1;
}

// The chunk kernels' block -> chunk map.  Workgroups go to the 8 XCDs round-robin
// (block b on XCD b % 8): each XCD gets a contiguous run of chunks instead, so a chunk's
// halo bytes are its neighbours' (the same L2) and each XCD streams its own region of
// the arena (r04: held-out mlm tokenize 2.33 -> 2.25 ms).  A bijection on [0, gridDim.x).
__device__ __forceinline__ int64_t xcd_chunk() {
    const int64_t G = gridDim.x, b = blockIdx.x, x = b & 7, q = G >> 3, rem = G & 7;
    return x * q + (x < rem ? x : rem) + (b >> 3);
}

}  // namespace sdl
