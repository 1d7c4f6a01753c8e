/*
 * orc_batcher.c -- CPU restatement of the reference Batcher stage (TEST
 * INFRASTRUCTURE ONLY: the checker for the HIP path and bench.py's CPU
 * baseline, never the product).
 *
 *   GenTokenizer           rust/src/tasks/gen_batcher.rs:44-98   (mlm, clm, span)
 *   SimpleBatcher          rust/src/models/simple_batcher.rs:35-53 (multi-label)
 *   BertData               rust/src/models/bert_data.rs:40-89    (Mask, MultiLabel)
 *   GptData                rust/src/models/gpt_data.rs:29-45
 *   T5Data (Span)          rust/src/models/t5_data.rs:162-226
 *   encode_mask framing    rust/src/tokenizer/tokenizer_wrapper.rs:107-134
 *   RNG contract           DESIGN.md §3 (replaces the unseedable thread_rng)
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "orc_internal.h"

/* ------------------------------------------------------------------------- */
/* RNG contract: Philox4x32-10 (Salmon et al., SC'11 / Random123)             */
/* ------------------------------------------------------------------------- */
static void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0;
        c[1] = lo1;
        c[2] = n2;
        c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

/* key(pos) = Philox(counter = (pos/4, chunk, rec_lo, rec_hi), key = seed)[pos%4] */
uint32_t orc_mlm_key(uint64_t seed, uint64_t record, uint32_t chunk, uint32_t pos) {
    uint32_t c[4] = {pos >> 2, chunk, (uint32_t)record, (uint32_t)(record >> 32)};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    return c[pos & 3];
}

/* ------------------------------------------------------------------------- */
/* Optional rand-compatible MLM mode (cfg.rng_mode = 1): BertData::mask_batch's */
/* `position_base.shuffle(&mut thread_rng())` (bert_data.rs:40-43) with        */
/* thread_rng replaced by a StdRng per row:                                     */
/*     StdRng::from_seed(row_seed)   row_seed = seed (u64 LE) | record (u64 LE) */
/*                                              | chunk (u32 LE) | 12 zero bytes */
/* restating, from their published sources (not vendored, not buildable here): */
/*   rand_chacha 0.3.1  StdRng = ChaCha12Rng: key = the 32-byte seed, 64-bit    */
/*                      block counter in words 12-13 from 0, stream 0 in words  */
/*                      14-15, output words in block order;                     */
/*   rand 0.8.5         SliceRandom::shuffle -> gen_index -> gen_range(0..n) ->   */
/*                      UniformInt<u32>::sample_single_inclusive (widening       */
/*                      multiply, zone = (range << lz(range)) - 1, rejection).    */
/* Pinned (tests/test_rand_mode.py) by RFC 7539's ChaCha20 vectors, rand's       */
/* test_stdrng_construction vectors and rand's value_stability_slice shuffle.   */
/* ------------------------------------------------------------------------- */
static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
#define ORC_QR(a, b, c, d)                                                      \
    a += b; d ^= a; d = rotl32(d, 16); c += d; b ^= c; b = rotl32(b, 12);       \
    a += b; d ^= a; d = rotl32(d, 8);  c += d; b ^= c; b = rotl32(b, 7);

void orc_chacha_block(const uint32_t key[8], uint64_t counter, uint64_t stream, int rounds, uint32_t out[16]) {
    const uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                            key[4], key[5], key[6], key[7], (uint32_t)counter, (uint32_t)(counter >> 32),
                            (uint32_t)stream, (uint32_t)(stream >> 32)};
    uint32_t x[16];
    memcpy(x, s, sizeof(x));
    for (int i = 0; i < rounds; i += 2) {
        ORC_QR(x[0], x[4], x[8], x[12]) ORC_QR(x[1], x[5], x[9], x[13])
        ORC_QR(x[2], x[6], x[10], x[14]) ORC_QR(x[3], x[7], x[11], x[15])
        ORC_QR(x[0], x[5], x[10], x[15]) ORC_QR(x[1], x[6], x[11], x[12])
        ORC_QR(x[2], x[7], x[8], x[13]) ORC_QR(x[3], x[4], x[9], x[14])
    }
    for (int i = 0; i < 16; ++i) out[i] = x[i] + s[i];
}

typedef struct {
    uint32_t key[8];
    uint64_t ctr;
    uint32_t buf[16];
    int idx;
} orc_stdrng;

static void stdrng_from_seed(orc_stdrng *r, const uint8_t seed[32]) {
    for (int i = 0; i < 8; ++i)
        r->key[i] = (uint32_t)seed[4 * i] | (uint32_t)seed[4 * i + 1] << 8 | (uint32_t)seed[4 * i + 2] << 16 |
                    (uint32_t)seed[4 * i + 3] << 24;
    r->ctr = 0;
    r->idx = 16;
}
static uint32_t stdrng_u32(orc_stdrng *r) {
    if (r->idx >= 16) {
        orc_chacha_block(r->key, r->ctr++, 0, 12, r->buf);
        r->idx = 0;
    }
    return r->buf[r->idx++];
}
/* first u64 of StdRng::from_seed(seed) (next_u64: low word first) -- for the KAT */
uint64_t orc_stdrng_first_u64(const uint8_t seed[32]) {
    orc_stdrng r;
    stdrng_from_seed(&r, seed);
    const uint64_t lo = stdrng_u32(&r);
    return lo | (uint64_t)stdrng_u32(&r) << 32;
}
/* gen_index(rng, n) = gen_range(0..n as u32) */
static uint32_t gen_index(orc_stdrng *r, uint32_t n) {
    const uint32_t zone = (n << __builtin_clz(n)) - 1u;
    for (;;) {
        const uint64_t m = (uint64_t)stdrng_u32(r) * n;
        if ((uint32_t)m <= zone) return (uint32_t)(m >> 32);
    }
}
/* position_base after `shuffle` with the row's StdRng */
void orc_rand_positions(uint64_t seed, uint64_t record, uint32_t chunk, int S, uint32_t *pos) {
    uint8_t sd[32] = {0};
    for (int b = 0; b < 8; ++b) {
        sd[b] = (uint8_t)(seed >> (8 * b));
        sd[8 + b] = (uint8_t)(record >> (8 * b));
    }
    for (int b = 0; b < 4; ++b) sd[16 + b] = (uint8_t)(chunk >> (8 * b));
    orc_stdrng r;
    stdrng_from_seed(&r, sd);
    for (int i = 0; i < S; ++i) pos[i] = (uint32_t)i;
    for (int i = S - 1; i >= 1; --i) {
        const uint32_t j = gen_index(&r, (uint32_t)i + 1u);
        const uint32_t t = pos[i];
        pos[i] = pos[j];
        pos[j] = t;
    }
}

/* ------------------------------------------------------------------------- */
/* Optional rand-compatible span mode (cfg.rng_mode = 1): T5Data::put_data's   */
/* random_data_gap / random_data_size (t5_data.rs:165-176) draw               */
/* `thread_rng().sample(StandardNormal)` as f64; with thread_rng replaced by   */
/* the row's StdRng (same row_seed as the MLM mode) they are, in order, gap    */
/* then size of pass 0, gap then size of pass 1, ...  Restated from the        */
/* published sources (not vendored, not buildable here):                        */
/*   rand_distr 0.4.3 StandardNormal for f64 = utils::ziggurat(rng, symmetric,  */
/*     ZIG_NORM_X, ZIG_NORM_F, pdf = exp(-x*x/2), zero_case): bits = next_u64; */
/*     i = bits & 0xff; u = f64 from bits>>12 with exponent 1, minus 3 ([-1,1));*/
/*     x = u * X[i]; |x| < X[i+1] -> x; i == 0 -> tail: x = ln(Open01)/R,       */
/*     y = ln(Open01) until -2y >= x*x, +-(R - x); else the wedge test          */
/*     F[i+1] + (F[i] - F[i+1]) * gen::<f64>() < pdf(x) -> x, else retry;      */
/*   the tables come from rand's ziggurat_tables.py (R = 3.6541528853610088,    */
/*     V = 0.00492867323399, 256 layers) printed with %.18f;                  */
/*   rand 0.8.5 Open01 (52-bit fraction in [1,2) minus 1 - EPSILON/2),          */
/*     Standard f64 ((next_u64 >> 11) * 2^-53).                               */
/* `distance as usize` saturates: NaN and negatives give 0.                    */
/* Pinned (tests/test_rand_mode.py) by rand_distr's value-stability vector for  */
/* StandardNormal (seed 213 of its Pcg32 test rng): -0.11844188827977231,      */
/* 0.7813779637772346, 0.06563993969580051, -1.1932899004186373.             */
/* ------------------------------------------------------------------------- */
#define ZIG_R 3.6541528853610088
static double ZX[257], ZF[257];
static void zig_tables(void) {
    static int init;
    if (init) return;
    const double V = 0.00492867323399;
    double x[257];
    x[0] = V / exp(-ZIG_R * ZIG_R / 2.0);
    x[1] = ZIG_R;
    for (int i = 2; i < 256; ++i) x[i] = sqrt(-2.0 * log(V / x[i - 1] + exp(-x[i - 1] * x[i - 1] / 2.0)));
    x[256] = 0.0;
    char buf[64];
    for (int i = 0; i < 257; ++i) { /* the Rust source holds the %.18f texts */
        snprintf(buf, sizeof buf, "%.18f", x[i]);
        ZX[i] = strtod(buf, NULL);
        snprintf(buf, sizeof buf, "%.18f", exp(-x[i] * x[i] / 2.0));
        ZF[i] = strtod(buf, NULL);
    }
    init = 1;
}
typedef uint64_t (*u64_source)(void *);
static double f64_bits(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
static double std_normal(u64_source next, void *st) {
    zig_tables();
    for (;;) {
        const uint64_t bits = next(st);
        const int i = (int)(bits & 0xff);
        const double u = f64_bits((bits >> 12) | (uint64_t)1024 << 52) - 3.0;
        const double x = u * ZX[i];
        if (fabs(x) < ZX[i + 1]) return x;
        if (i == 0) { /* zero_case: the tail beyond R */
            double xt = 1.0, yt = 0.0;
            while (-2.0 * yt < xt * xt) {
                const double a = f64_bits((next(st) >> 12) | (uint64_t)1023 << 52) - (1.0 - DBL_EPSILON / 2.0);
                const double c = f64_bits((next(st) >> 12) | (uint64_t)1023 << 52) - (1.0 - DBL_EPSILON / 2.0);
                xt = log(a) / ZIG_R;
                yt = log(c);
            }
            return u < 0.0 ? xt - ZIG_R : ZIG_R - xt;
        }
        const double g = (double)(next(st) >> 11) * (1.0 / 9007199254740992.0);
        if (ZF[i + 1] + (ZF[i] - ZF[i + 1]) * g < exp(-x * x / 2.0)) return x;
    }
}
static uint64_t stdrng_u64(void *r) { /* BlockRng::next_u64 at an even index: low word first */
    const uint64_t lo = stdrng_u32((orc_stdrng *)r);
    return lo | (uint64_t)stdrng_u32((orc_stdrng *)r) << 32;
}
/* rand_pcg 0.3 Pcg32::new(state, stream) (Lcg64Xsh32), next_u64 = two next_u32, low first */
typedef struct { uint64_t state, inc; } orc_pcg32;
static uint32_t pcg32_u32(orc_pcg32 *p) {
    const uint64_t s = p->state;
    p->state = s * 6364136223846793005ull + p->inc;
    const uint32_t rot = (uint32_t)(s >> 59), xsh = (uint32_t)(((s >> 18) ^ s) >> 27);
    return (xsh >> rot) | (xsh << ((32 - rot) & 31));
}
static uint64_t pcg32_u64(void *p) {
    const uint64_t lo = pcg32_u32((orc_pcg32 *)p);
    return lo | (uint64_t)pcg32_u32((orc_pcg32 *)p) << 32;
}
/* n StandardNormal f64 samples from Pcg32::new(state, stream) -- for the KAT */
void orc_normal_pcg32(uint64_t state, uint64_t stream, int n, double *out) {
    orc_pcg32 p = {0, (stream << 1) | 1u};
    p.state = state + p.inc;
    p.state = p.state * 6364136223846793005ull + p.inc;
    for (int k = 0; k < n; ++k) out[k] = std_normal(pcg32_u64, &p);
}
/* n StandardNormal f64 samples from the row's StdRng (the span mode's stream) */
static void row_stdrng(orc_stdrng *r, uint64_t seed, uint64_t record, uint32_t chunk) {
    uint8_t sd[32] = {0};
    for (int b = 0; b < 8; ++b) {
        sd[b] = (uint8_t)(seed >> (8 * b));
        sd[8 + b] = (uint8_t)(record >> (8 * b));
    }
    for (int b = 0; b < 4; ++b) sd[16 + b] = (uint8_t)(chunk >> (8 * b));
    stdrng_from_seed(r, sd);
}
void orc_normal_row(uint64_t seed, uint64_t record, uint32_t chunk, int n, double *out) {
    orc_stdrng r;
    row_stdrng(&r, seed, record, chunk);
    for (int k = 0; k < n; ++k) out[k] = std_normal(stdrng_u64, &r);
}
/* `f as usize` (Rust saturating float -> int cast) */
static size_t sat_usize(double d) {
    if (!(d > 0.0)) return 0; /* NaN, negatives, -0.0 */
    if (d >= 18446744073709551616.0) return SIZE_MAX;
    return (size_t)d;
}

/* Span draws: the reference's trunc(avg - z) with z ~ StandardNormal
 * (t5_data.rs:165-176, `as usize` saturating at 0) is sampled exactly in
 * distribution by inverting its CDF on a 32-bit uniform:
 *   P(v <= k) = P(z > avg - k - 1) = erfc((avg - k - 1) / sqrt 2) / 2,
 *   thr[j] = floor(2^32 P(v <= kmin + j)),  v = kmin + #{j : thr[j] <= x}.
 * `lo` is the smallest value v can take (0 for the gap; 1 for the size, whose
 * max(.., 1) folds everything below into 1). */
void orc_span_table(double avg, int lo, int32_t *kmin, int32_t *n, uint32_t *thr, int cap) {
    double k0 = floor(avg - 10.0);
    if (k0 < lo) k0 = lo;
    if (k0 > 1e9) k0 = 1e9;
    *kmin = (int32_t)k0;
    int m = 0;
    for (int j = 0; j < cap; ++j) {
        const double cdf = 0.5 * erfc((avg - (k0 + j) - 1.0) / sqrt(2.0));
        const double t = floor(cdf * 4294967296.0);
        if (t >= 4294967296.0) break;
        thr[m++] = (uint32_t)t;
    }
    *n = m;
}

/* The two uniforms of span pass `pass` of row (record, chunk). */
static void span_draws(uint64_t seed, uint64_t rec, uint32_t chunk, uint32_t pass, uint32_t *xg, uint32_t *xs) {
    uint32_t c[4] = {pass, chunk | 0x40000000u, (uint32_t)rec, (uint32_t)(rec >> 32)};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    *xg = c[0];
    *xs = c[1];
}
static uint32_t span_pick(const int32_t kmin, const int32_t n, const uint32_t *thr, uint32_t x) {
    int32_t v = kmin;
    for (int j = 0; j < n; ++j) v += thr[j] <= x;
    return (uint32_t)v;
}

/* ------------------------------------------------------------------------- */
/* DataSet                                                                    */
/* ------------------------------------------------------------------------- */
typedef struct {
    int32_t *ids, *am, *tt, *lab; /* [B,S] x3, [B,LW] */
    float *f32;                   /* [B,NL] (multi-label) */
    int index;
} obatch;

#define SPAN_TAB 32
struct orc_batcher {
    orc_encoder enc;
    orc_cfg c;
    int LW, NL;
    int32_t gap_kmin, gap_n, size_kmin, size_n;
    uint32_t gap_thr[SPAN_TAB], size_thr[SPAN_TAB];
    uint64_t span_errors; /* label/sentinel writes the reference would panic on */
    uint64_t n_records;
    obatch **q;
    int qh, qn, qcap;
};

/* BertData::new / GptData::new: BatchConfig::create_vector (batcher.rs:17-22):
 * input_ids 0, attention_mask 1, token_type_ids 0, labels -100 (GptData) --
 * BertData's labels are pushed per row and have no initial value; the ABI
 * reports them as -100 past `rows`. */
static obatch *obatch_new(const orc_batcher *b) {
    obatch *x = (obatch *)calloc(1, sizeof(obatch));
    size_t bs = (size_t)b->c.B * b->c.S, bl = (size_t)b->c.B * b->LW;
    x->ids = (int32_t *)calloc(bs, 4);
    x->am = (int32_t *)malloc(bs * 4);
    x->tt = (int32_t *)calloc(bs, 4);
    x->lab = (int32_t *)malloc((bl ? bl : 1) * 4);
    x->f32 = (float *)calloc((size_t)b->c.B * (b->NL ? b->NL : 1), 4);
    for (size_t i = 0; i < bs; ++i) x->am[i] = 1;
    for (size_t i = 0; i < bl; ++i) x->lab[i] = -100;
    return x;
}

static void obatch_free(obatch *x) {
    free(x->ids);
    free(x->am);
    free(x->tt);
    free(x->lab);
    free(x->f32);
    free(x);
}

static void q_push(orc_batcher *b, obatch *x) {
    if (b->qh + b->qn == b->qcap) {
        if (b->qh) {
            memmove(b->q, b->q + b->qh, sizeof(obatch *) * b->qn);
            b->qh = 0;
        } else {
            b->qcap = b->qcap ? 2 * b->qcap : 8;
            b->q = (obatch **)realloc(b->q, sizeof(obatch *) * b->qcap);
        }
    }
    b->q[b->qh + b->qn++] = x;
}

orc_batcher *orc_batcher_create(const orc_encoder *e, const orc_cfg *c) {
    if (!e || !c || c->B <= 0 || c->S <= 0) return NULL;
    if (c->task != ORC_MLM && c->task != ORC_CLM && c->task != ORC_MULTI_LABEL && c->task != ORC_SPAN &&
        c->task != ORC_SINGLE_CLASS)
        return NULL;
    if (c->task == ORC_SPAN && c->S < 4) return NULL;
    if (c->task == ORC_MLM && (c->mask_length < 0 || c->mask_length > c->S)) return NULL;
    if (c->task == ORC_MULTI_LABEL && c->number_labels <= 0) return NULL;
    orc_batcher *b = (orc_batcher *)calloc(1, sizeof(orc_batcher));
    b->enc = *e;
    b->c = *c;
    if (c->task == ORC_MULTI_LABEL || c->task == ORC_SINGLE_CLASS) { /* SimpleBatcher: no chunking, no filter */
        b->c.chunk = 0;
        b->c.min_ids = 0;
    }
    b->NL = c->task == ORC_MULTI_LABEL ? c->number_labels : 0;
    b->LW = c->task == ORC_MULTI_LABEL ? 0 : c->task == ORC_SINGLE_CLASS ? 1 : c->task == ORC_SPAN ? c->S / 4 : c->S;
    /* t5_data.rs:44 for span; SingleClass: one u32 per row */
    if (c->task == ORC_SPAN) {
        orc_span_table(c->avg_span_gap, 0, &b->gap_kmin, &b->gap_n, b->gap_thr, SPAN_TAB);
        orc_span_table(c->avg_span_size, 1, &b->size_kmin, &b->size_n, b->size_thr, SPAN_TAB);
    }
    q_push(b, obatch_new(b)); /* GenTokenizer::new / SimpleBatcher::new: first DataSet */
    return b;
}

typedef struct { uint32_t key, pos; } kp;
static int kp_cmp(const void *a, const void *b) {
    const kp *x = (const kp *)a, *y = (const kp *)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->pos < y->pos ? -1 : (x->pos > y->pos);
}

/* BertData::mask_batch (bert_data.rs:40-53) under the RNG contract: the first
 * mask_length entries of the shuffled positions are the mask_length smallest
 * (key, position) pairs. */
static void mask_row(const orc_batcher *b, int32_t *in, int32_t *lb, uint64_t rec, uint32_t chunk) {
    const int S = b->c.S;
    if (b->c.rng_mode == 1) { /* rand-compatible mode: the shuffled positions themselves */
        uint32_t *pos = (uint32_t *)malloc(sizeof(uint32_t) * S);
        orc_rand_positions(b->c.seed, rec, chunk, S, pos);
        for (int j = 0; j < S; ++j) lb[j] = -100;
        for (int k = 0; k < b->c.mask_length; ++k) {
            const uint32_t p = pos[k];
            if (in[p] != 0) {
                lb[p] = in[p];
                in[p] = b->c.mask_id;
            }
        }
        free(pos);
        return;
    }
    kp *perm = (kp *)malloc(sizeof(kp) * S);
    for (int p = 0; p < S; ++p) {
        perm[p].key = orc_mlm_key(b->c.seed, rec, chunk, (uint32_t)p);
        perm[p].pos = (uint32_t)p;
    }
    qsort(perm, (size_t)S, sizeof(kp), kp_cmp);
    for (int j = 0; j < S; ++j) lb[j] = -100;
    for (int k = 0; k < b->c.mask_length; ++k) {
        uint32_t p = perm[k].pos;
        if (in[p] != 0) {
            lb[p] = in[p];
            in[p] = b->c.mask_id;
        }
    }
    free(perm);
}

/* DataSet::put_full_data for one row (dataset.rs:47-61).  Returns -1 on a
 * label index >= number_labels (the reference panics: bert_data.rs:70-72). */
static int put_data(orc_batcher *b, obatch *x, const uint32_t *ids, size_t n, uint64_t rec, uint32_t chunk,
                    const uint32_t *labels, size_t nl) {
    const size_t S = (size_t)b->c.S;
    int32_t *in = x->ids + (size_t)x->index * S;
    int32_t *am = x->am + (size_t)x->index * S;
    const size_t l = n < S ? n : S;
    for (size_t j = 0; j < l; ++j) in[j] = (int32_t)ids[j];
    switch (b->c.task) {
    case ORC_MLM:
    case ORC_SINGLE_CLASS:
    case ORC_MULTI_LABEL: /* BertData::put_data (bert_data.rs:55-89) */
        if (n < S)
            for (size_t j = S - n; j < S; ++j) am[j] = 0; /* reversed-range quirk */
        if (b->c.task == ORC_MLM) {
            mask_row(b, in, x->lab + (size_t)x->index * S, rec, chunk);
        } else if (b->c.task == ORC_SINGLE_CLASS) {
            /* label.map(|s| self.label.push(s)) (bert_data.rs:79-81); SingleClassArrowGenerator
             * always yields Some(Label::Single) (single_arrow.rs:16-26): exactly one label */
            if (nl != 1) return -1;
            x->lab[x->index] = (int32_t)labels[0];
        } else {
            float *f = x->f32 + (size_t)x->index * b->NL;
            for (size_t k = 0; k < nl; ++k) {
                if (labels[k] >= (uint32_t)b->NL) return -1;
                f[labels[k]] = 1.0f;
            }
        }
        break;
    case ORC_SPAN: { /* T5Data::put_data (t5_data.rs:162-226), one chunk = one row */
        int32_t *lb = x->lab + (size_t)x->index * b->LW;
        const size_t LW = (size_t)b->LW;
        for (size_t j = 0; j < l; ++j) in[j] = 0; /* rewritten below */
        size_t ip = 0, lp = 0, ap = 0;
        uint32_t pass = 0;
        const int rnd = b->c.rng_mode == 1;
        orc_stdrng rr;
        if (rnd) row_stdrng(&rr, b->c.seed, rec, chunk);
#define EXTRA(k) ((k) < 100 ? (int32_t)b->enc.extra[k] : (b->span_errors++, (int32_t)b->enc.extra[99]))
#define LAB(i, v) do { if ((i) < LW) lb[i] = (v); else b->span_errors++; } while (0)
        while (lp < S) {
            uint32_t xg = 0, xs = 0;
            if (!rnd) span_draws(b->c.seed, rec, chunk, pass, &xg, &xs);
            size_t g = rnd ? sat_usize(b->c.avg_span_gap - std_normal(stdrng_u64, &rr))
                           : span_pick(b->gap_kmin, b->gap_n, b->gap_thr, xg);
            if (g > S - lp) g = S - lp;
            if (g > n - ip) g = n - ip;
            for (size_t j = 0; j < g; ++j) in[lp + j] = (int32_t)ids[ip + j];
            lp += g;
            ip += g;
            size_t sz;
            if (rnd) {
                sz = sat_usize(b->c.avg_span_size - std_normal(stdrng_u64, &rr));
                if (sz < 1) sz = 1; /* std::cmp::max(distance as usize, 1) */
            } else {
                sz = span_pick(b->size_kmin, b->size_n, b->size_thr, xs);
            }
            if (sz > S - lp) sz = S - lp;
            if (sz > n - ip) sz = n - ip;
            if (sz > 0) {
                const int32_t e = EXTRA(pass);
                in[lp] = e;
                LAB(ap, e);
                for (size_t j = 0; j < sz; ++j) LAB(ap + j + 1, (int32_t)ids[ip + j]);
                lp += 1;
                ip += sz;
                ap += sz + 1;
            }
            if (n <= ip) { /* attention_mask untouched: the loop 0..ip-n is empty */
                const int32_t e2 = EXTRA(pass + 1); /* Rust evaluates the right-hand side first */
                LAB(ap, e2);
                break;
            }
            pass++;
        }
#undef EXTRA
#undef LAB
        break;
    }
    case ORC_CLM: { /* GptData::put_data (gpt_data.rs:29-45): labels = row, no shift */
        int32_t *lb = x->lab + (size_t)x->index * S;
        for (size_t j = 0; j < S; ++j) lb[j] = in[j];
        if (n < S)
            for (size_t j = S - n; j < S; ++j) {
                lb[j] = -100;
                am[j] = 0;
            }
        break;
    }
    }
    x->index++;
    return 0;
}

static void batch_out(const orc_batcher *b, obatch *x, orc_out *o) {
    if (o) {
        size_t bs = (size_t)b->c.B * b->c.S;
        if (o->ids) memcpy(o->ids, x->ids, bs * 4);
        if (o->am) memcpy(o->am, x->am, bs * 4);
        if (o->tt) memcpy(o->tt, x->tt, bs * 4);
        if (o->lab && b->LW) memcpy(o->lab, x->lab, (size_t)b->c.B * b->LW * 4);
        if (o->f32 && b->NL) memcpy(o->f32, x->f32, (size_t)b->c.B * b->NL * 4);
        o->rows = x->index;
    }
    obatch_free(x);
}

static obatch *q_pop(orc_batcher *b) {
    obatch *x = b->q[b->qh];
    b->qh++;
    b->qn--;
    return x;
}

int orc_batcher_push_ex(orc_batcher *b, const uint8_t *s, size_t n, const uint32_t *labels, size_t nl,
                        orc_out *out) {
    const uint64_t rec = b->n_records++;
    idvec v = {0};
    for (int i = 0; i < b->enc.npre; ++i) idpush(&v, b->enc.pre[i]);
    b->enc.encode(b->enc.impl, s, n, &v);
    for (int i = 0; i < b->enc.npost; ++i) idpush(&v, b->enc.post[i]);
    if (v.n < (size_t)b->c.min_ids) { /* gen_batcher.rs:74-76 */
        free(v.p);
        return 0;
    }
    const size_t step = b->c.chunk ? (size_t)b->c.S : (v.n ? v.n : 1);
    uint32_t chunk = 0;
    int rc = 0;
    for (size_t off = 0; off < v.n || (off == 0 && v.n == 0); off += step, ++chunk) { /* chunks_mut(S) */
        size_t len = v.n - off < step ? v.n - off : step;
        obatch *back = b->q[b->qh + b->qn - 1];
        if (put_data(b, back, v.p + off, len, rec, chunk, labels, nl)) rc = -1; /* handle_internal_batch */
        if (back->index == b->c.B) q_push(b, obatch_new(b));
        if (v.n == 0) break;
    }
    free(v.p);
    if (rc) return rc;
    if (b->q[b->qh]->index == b->c.B) { /* gen_batcher.rs:86-91 / simple_batcher.rs:39-41 */
        batch_out(b, q_pop(b), out);
        return 1;
    }
    return 0;
}

int orc_batcher_flush_ex(orc_batcher *b, orc_out *out) {
    if (b->c.task == ORC_MULTI_LABEL || b->c.task == ORC_SINGLE_CLASS) { /* SimpleBatcher::get_working_batch */
        batch_out(b, q_pop(b), out);
        q_push(b, obatch_new(b));
        return 1;
    }
    if (b->qn == 0) return 0; /* GenTokenizer::get_working_batch = store.pop_front() */
    batch_out(b, q_pop(b), out);
    return 1;
}

void orc_batcher_free(orc_batcher *b) {
    for (int i = 0; i < b->qn; ++i) obatch_free(b->q[b->qh + i]);
    free(b->q);
    free(b);
}

void orc_batcher_set_next_record(orc_batcher *b, uint64_t record) { b->n_records = record; }
uint64_t orc_batcher_span_errors(const orc_batcher *b) { return b->span_errors; }

/* ---- round-1 MLM entry points (4 planes [B,S] back to back) ---- */
orc_batcher *orc_batcher_new(const orc_tok *t, int task, int batch_size, int seq_len, int mask_length, int mask_id,
                             uint64_t seed) {
    if (task != ORC_MLM) return NULL;
    orc_encoder e;
    orc_encoder_bert(t, &e);
    orc_cfg c;
    orc_cfg_default(&c, task);
    c.B = batch_size;
    c.S = seq_len;
    c.mask_length = mask_length;
    c.mask_id = mask_id;
    c.seed = seed;
    return orc_batcher_create(&e, &c);
}

static void planes_out(const orc_batcher *b, int32_t *out, orc_out *o) {
    size_t bs = (size_t)b->c.B * b->c.S;
    memset(o, 0, sizeof(*o));
    if (out) {
        o->ids = out;
        o->am = out + bs;
        o->tt = out + 2 * bs;
        o->lab = out + 3 * bs;
    }
}

int orc_batcher_push(orc_batcher *b, const uint8_t *s, size_t n, int32_t *out, int *rows) {
    orc_out o;
    planes_out(b, out, &o);
    int r = orc_batcher_push_ex(b, s, n, NULL, 0, &o);
    if (r == 1 && rows) *rows = o.rows;
    return r;
}

int orc_batcher_flush(orc_batcher *b, int32_t *out, int *rows) {
    orc_out o;
    planes_out(b, out, &o);
    int r = orc_batcher_flush_ex(b, &o);
    if (r == 1 && rows) *rows = o.rows;
    return r;
}

void orc_batcher_set_rng_mode(orc_batcher *b, int mode) { b->c.rng_mode = mode; }

void orc_cfg_default(orc_cfg *c, int task) {
    memset(c, 0, sizeof(*c));
    c->task = task;
    c->B = 4096;
    c->S = 128;
    c->chunk = task == ORC_MULTI_LABEL || task == ORC_SINGLE_CLASS ? 0 : 1;
    c->min_ids = task == ORC_MULTI_LABEL || task == ORC_SINGLE_CLASS ? 0 : 64;
    c->mask_length = (int)((float)c->S * 0.15f);
    c->mask_id = 103;
    c->number_labels = 9;
    c->avg_span_gap = 16.0;
    c->avg_span_size = 2.0;
}

size_t orc_encoder_size(void) { return sizeof(orc_encoder); }
