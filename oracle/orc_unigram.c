/*
 * orc_unigram.c -- CPU restatement of the t5-small tokenizer (TEST
 * INFRASTRUCTURE ONLY: the checker for the HIP path, never the product).
 *
 * What the reference calls for task=span: TokenizerHolder::get_ids ->
 * tokenizers::Tokenizer::encode(text, true) (rust/src/tokenizer/tokenizer_holder.rs:19-28;
 * crate tokenizers 0.13.1, not vendored) with the hub's t5-small tokenizer.json
 * (name at rust/src/tasks/masking/masking_cases.rs:80):
 *   AddedVocabulary split: <pad> </s> <unk> <extra_id_0..99>, leftmost-longest
 *     on the raw text (tokenizer/added_vocabulary.rs);
 *   -> Precompiled normalizer (normalizers/precompiled.rs + crate
 *      spm_precompiled): the segment is cut into extended grapheme clusters
 *      (crate unicode-segmentation, UAX #29); a cluster of < 6 bytes whose
 *      bytes have a charsmap key as prefix becomes the normalized string of
 *      the SHORTEST such key; otherwise each char is looked up the same way
 *      and kept when no key is a prefix of it;
 *   -> WhitespaceSplit (char::is_whitespace, removed);
 *   -> Metaspace("▁", add_prefix_space): "▁" prepended unless the word starts
 *      with it, split before every "▁" (MergedWithNext);
 *   -> Unigram (models/unigram/model.rs encode_optimized): Viterbi over char
 *      boundaries, candidates = every vocab piece that is a prefix at the
 *      start (shortest first), replaced only by a strictly better f64 score;
 *      a char start with no one-char piece also offers [unk] with score
 *      min_score - 10; consecutive [unk] nodes are fused into one string;
 *      each string -> its id, else unk_id;
 *   -> TemplateProcessing "$A </s>".
 * Then TokenizerWrapper::encode_mask for T5: [</s>] + ids + [</s>]
 * (tokenizer_wrapper.rs:125-131).
 *
 * The grapheme-cluster properties come from data/t5_graphemes.bin
 * (tools/make_t5_tables.py); the charsmap trie is read from the
 * tokenizer.json.  Input that is not valid UTF-8 cannot reach the reference
 * (a Rust String); here an invalid byte is one U+FFFD char (its 3 bytes).
 */
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "orc_internal.h"
#include "orc_json.h"

enum { G_OTHER = 0, G_CR, G_LF, G_CONTROL, G_EXTEND, G_ZWJ, G_RI, G_PREPEND, G_SPACING, G_L, G_V, G_T, G_LV, G_LVT };
#define P_EXTPICT 0x10u
#define P_WS 0x80u
#define INCB(p) (((p) >> 5) & 3u) /* 1 Linker 2 Consonant 3 Extend */

#define MAX_SPECIAL_T5 128

typedef struct {
    char **keys;
    size_t *lens;
    int *vals;
    size_t cap;
} vmap;

static uint64_t vh(const uint8_t *p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}
static int vmap_get(const vmap *m, const uint8_t *k, size_t n) {
    for (size_t i = vh(k, n) & (m->cap - 1);; i = (i + 1) & (m->cap - 1)) {
        if (!m->keys[i]) return -1;
        if (m->lens[i] == n && !memcmp(m->keys[i], k, n)) return m->vals[i];
    }
}
static void vmap_put(vmap *m, const uint8_t *k, size_t n, int v) {
    for (size_t i = vh(k, n) & (m->cap - 1);; i = (i + 1) & (m->cap - 1)) {
        if (!m->keys[i]) {
            m->keys[i] = (char *)malloc(n + 1);
            memcpy(m->keys[i], k, n);
            m->lens[i] = n;
            m->vals[i] = v;
            return;
        }
        if (m->lens[i] == n && !memcmp(m->keys[i], k, n)) { m->vals[i] = v; return; }
    }
}

struct orc_t5 {
    vmap vocab;
    double *score;
    int n_vocab, unk_id, eos_id, max_piece;
    double unk_score;
    uint32_t *units; /* charsmap double array */
    size_t n_units;
    char *norm;      /* normalized strings, NUL separated */
    size_t norm_len;
    uint8_t *prop;   /* 0x110000 grapheme/whitespace properties */
    int n_special;
    char *special[MAX_SPECIAL_T5];
    size_t special_len[MAX_SPECIAL_T5];
    int special_id[MAX_SPECIAL_T5];
};

static char *slurp(const char *path, size_t *n) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *b = (char *)malloc((size_t)sz + 1);
    if (fread(b, 1, (size_t)sz, f) != (size_t)sz) { fclose(f); free(b); return NULL; }
    fclose(f);
    *n = (size_t)sz;
    return b;
}

static int b64v(int c) {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+') return 62;
    if (c == '/') return 63;
    return -1;
}
static uint8_t *b64dec(const char *s, size_t n, size_t *out_n) {
    uint8_t *o = (uint8_t *)malloc(n / 4 * 3 + 3);
    size_t k = 0;
    uint32_t acc = 0;
    int bits = 0;
    for (size_t i = 0; i < n; ++i) {
        int v = b64v((unsigned char)s[i]);
        if (v < 0) continue; /* '=' padding */
        acc = acc << 6 | (uint32_t)v;
        bits += 6;
        if (bits >= 8) { bits -= 8; o[k++] = (uint8_t)(acc >> bits); }
    }
    *out_n = k;
    return o;
}

static int load_props(orc_t5 *t, const char *path) {
    size_t n;
    char *b = slurp(path, &n);
    if (!b || n < 16 || memcmp(b, "SDLU", 4)) { free(b); return -1; }
    uint32_t ver, np, nb;
    memcpy(&ver, b + 4, 4);
    memcpy(&np, b + 8, 4);
    memcpy(&nb, b + 12, 4);
    if (ver != 1 || np != 0x110000 / 256 || n != 16 + 2 * (size_t)np + 256 * (size_t)nb) { free(b); return -1; }
    t->prop = (uint8_t *)malloc(0x110000);
    const uint16_t *page = (const uint16_t *)(b + 16);
    const uint8_t *blk = (const uint8_t *)(b + 16 + 2 * np);
    for (uint32_t cp = 0; cp < 0x110000; ++cp) t->prop[cp] = blk[(size_t)page[cp >> 8] * 256 + (cp & 255)];
    free(b);
    return 0;
}

void orc_t5_free(orc_t5 *t) {
    if (!t) return;
    if (t->vocab.keys) {
        for (size_t i = 0; i < t->vocab.cap; ++i) free(t->vocab.keys[i]);
        free(t->vocab.keys);
        free(t->vocab.lens);
        free(t->vocab.vals);
    }
    free(t->score);
    free(t->units);
    free(t->norm);
    free(t->prop);
    for (int i = 0; i < t->n_special; ++i) free(t->special[i]);
    free(t);
}

orc_t5 *orc_t5_load(const char *tokenizer_json, const char *graphemes_bin) {
    size_t n;
    char *body = slurp(tokenizer_json, &n);
    if (!body) return NULL;
    oj *root = oj_parse(body, n);
    free(body);
    if (!root) return NULL;
    orc_t5 *t = (orc_t5 *)calloc(1, sizeof(orc_t5));
    const oj *model = oj_get(root, "model");
    const oj *vocab = model ? oj_get(model, "vocab") : NULL, *unk = model ? oj_get(model, "unk_id") : NULL;
    const oj *nz = oj_get(root, "normalizer");
    const oj *cm = nz ? oj_get(nz, "precompiled_charsmap") : NULL;
    if (!vocab || vocab->kind != OJ_ARR || !unk || !cm || cm->kind != OJ_STR || load_props(t, graphemes_bin)) goto fail;
    t->n_vocab = (int)vocab->n;
    t->unk_id = (int)unk->num;
    t->vocab.cap = 16;
    while (t->vocab.cap < 2 * vocab->n + 16) t->vocab.cap <<= 1;
    t->vocab.keys = (char **)calloc(t->vocab.cap, sizeof(char *));
    t->vocab.lens = (size_t *)calloc(t->vocab.cap, sizeof(size_t));
    t->vocab.vals = (int *)calloc(t->vocab.cap, sizeof(int));
    t->score = (double *)malloc(vocab->n * sizeof(double));
    double min_score = INFINITY;
    for (size_t i = 0; i < vocab->n; ++i) {
        const oj *e = &vocab->items[i];
        if (e->kind != OJ_ARR || e->n != 2 || e->items[0].kind != OJ_STR) goto fail;
        vmap_put(&t->vocab, (const uint8_t *)e->items[0].str, e->items[0].slen, (int)i);
        t->score[i] = e->items[1].num;
        if (t->score[i] < min_score) min_score = t->score[i];
        if ((int)e->items[0].slen > t->max_piece) t->max_piece = (int)e->items[0].slen;
    }
    t->unk_score = min_score - 10.0;
    size_t cmn;
    uint8_t *cmb = b64dec(cm->str, cm->slen, &cmn);
    uint32_t tsize;
    if (cmn < 4) { free(cmb); goto fail; }
    memcpy(&tsize, cmb, 4);
    if (4 + (size_t)tsize > cmn) { free(cmb); goto fail; }
    t->n_units = tsize / 4;
    t->units = (uint32_t *)malloc(tsize);
    memcpy(t->units, cmb + 4, tsize);
    t->norm_len = cmn - 4 - tsize;
    t->norm = (char *)malloc(t->norm_len + 1);
    memcpy(t->norm, cmb + 4 + tsize, t->norm_len);
    t->norm[t->norm_len] = 0;
    free(cmb);
    const oj *added = oj_get(root, "added_tokens");
    t->eos_id = -1;
    for (size_t i = 0; added && i < added->n && t->n_special < MAX_SPECIAL_T5; ++i) {
        const oj *c = oj_get(&added->items[i], "content"), *id = oj_get(&added->items[i], "id");
        if (!c || !id) continue;
        t->special[t->n_special] = (char *)malloc(c->slen + 1);
        memcpy(t->special[t->n_special], c->str, c->slen + 1);
        t->special_len[t->n_special] = c->slen;
        t->special_id[t->n_special] = (int)id->num;
        if (!strcmp(c->str, "</s>")) t->eos_id = (int)id->num;
        t->n_special++;
    }
    oj_free(root);
    if (t->eos_id < 0) { orc_t5_free(t); return NULL; }
    return t;
fail:
    oj_free(root);
    orc_t5_free(t);
    return NULL;
}

int orc_t5_eos(const orc_t5 *t) { return t->eos_id; }
int orc_t5_special_id(const orc_t5 *t, const char *s) {
    for (int i = 0; i < t->n_special; ++i)
        if (!strcmp(t->special[i], s)) return t->special_id[i];
    return -1;
}

/* ---- UTF-8 --------------------------------------------------------------- */
/* Length of the valid UTF-8 char at s[i] (1..4), 0 if the byte starts no
 * valid char (then it stands for U+FFFD). */
static int u8len(const uint8_t *s, size_t n, size_t i, uint32_t *cp) {
    uint8_t b = s[i];
    if (b < 0x80) { *cp = b; return 1; }
    int len;
    uint32_t c, min;
    if ((b & 0xE0) == 0xC0) { len = 2; c = b & 0x1F; min = 0x80; }
    else if ((b & 0xF0) == 0xE0) { len = 3; c = b & 0x0F; min = 0x800; }
    else if ((b & 0xF8) == 0xF0) { len = 4; c = b & 0x07; min = 0x10000; }
    else return 0;
    if (i + (size_t)len > n) return 0;
    for (int k = 1; k < len; ++k) {
        if ((s[i + k] & 0xC0) != 0x80) return 0;
        c = c << 6 | (s[i + k] & 0x3F);
    }
    if (c < min || c > 0x10FFFF || (c >= 0xD800 && c <= 0xDFFF)) return 0;
    *cp = c;
    return len;
}

/* Valid UTF-8 copy of s[0..n): invalid bytes -> U+FFFD. */
static uint8_t *sanitize(const uint8_t *s, size_t n, size_t *out_n) {
    uint8_t *o = (uint8_t *)malloc(3 * n + 1);
    size_t k = 0;
    for (size_t i = 0; i < n;) {
        uint32_t cp;
        int l = u8len(s, n, i, &cp);
        if (l == 0) { o[k++] = 0xEF; o[k++] = 0xBF; o[k++] = 0xBD; i += 1; continue; }
        memcpy(o + k, s + i, (size_t)l);
        k += (size_t)l;
        i += (size_t)l;
    }
    *out_n = k;
    return o;
}

/* ---- UAX #29 extended grapheme clusters ------------------------------------ */
typedef struct {
    uint8_t prev;   /* properties of the previous char */
    uint8_t ri_odd; /* the run of RI chars ending at prev has odd length */
    uint8_t ep_ext; /* prev ends ExtPict Extend* */
    uint8_t ep_zwj; /* prev is the ZWJ of ExtPict Extend* ZWJ */
    uint8_t incb;   /* 1: Consonant [Extend|Linker]*, 2: ... with a Linker */
} gstate;

/* Is there a cluster boundary before a char with properties p?  Updates s. */
int orc_gcb_break(void *state, uint32_t p_in) {
    gstate *s = (gstate *)state;
    const uint8_t p = (uint8_t)p_in;
    const uint32_t a = s->prev & 15u, b = p & 15u;
    int brk;
    if (a == G_CR && b == G_LF) brk = 0;                                                      /* GB3 */
    else if (a == G_CONTROL || a == G_CR || a == G_LF) brk = 1;                               /* GB4 */
    else if (b == G_CONTROL || b == G_CR || b == G_LF) brk = 1;                               /* GB5 */
    else if (a == G_L && (b == G_L || b == G_V || b == G_LV || b == G_LVT)) brk = 0;          /* GB6 */
    else if ((a == G_LV || a == G_V) && (b == G_V || b == G_T)) brk = 0;                      /* GB7 */
    else if ((a == G_LVT || a == G_T) && b == G_T) brk = 0;                                   /* GB8 */
    else if (b == G_EXTEND || b == G_ZWJ) brk = 0;                                            /* GB9 */
    else if (b == G_SPACING) brk = 0;                                                         /* GB9a */
    else if (a == G_PREPEND) brk = 0;                                                         /* GB9b */
    else if (INCB(p) == 2 && s->incb == 2) brk = 0;                                           /* GB9c */
    else if (a == G_ZWJ && s->ep_zwj && (p & P_EXTPICT)) brk = 0;                             /* GB11 */
    else if (a == G_RI && b == G_RI && s->ri_odd) brk = 0;                                    /* GB12/13 */
    else brk = 1;                                                                             /* GB999 */
    /* state after this char */
    s->ri_odd = b == G_RI ? (uint8_t)(a == G_RI ? !s->ri_odd : 1) : 0;
    const uint8_t ep_ext = (p & P_EXTPICT) ? 1 : (b == G_EXTEND && s->ep_ext) ? 1 : 0;
    s->ep_zwj = (uint8_t)(b == G_ZWJ && s->ep_ext);
    s->ep_ext = ep_ext;
    const uint32_t ic = INCB(p);
    s->incb = ic == 2 ? 1 : (s->incb && ic == 1) ? 2 : (s->incb && ic == 3) ? s->incb : 0;
    s->prev = p;
    return brk;
}
size_t orc_gcb_state_size(void) { return sizeof(gstate); }
/* starts a segment: the first char never breaks */
void orc_gcb_reset(void *state) { memset(state, 0, sizeof(gstate)); ((gstate *)state)->prev = G_CONTROL; }

uint32_t orc_t5_prop(const orc_t5 *t, uint32_t cp) { return cp < 0x110000 ? t->prop[cp] : 0; }

/* ---- charsmap trie (darts-clone double array, spm_precompiled) ------------- */
static inline uint32_t du_off(uint32_t u) { return (u >> 10) << ((u & (1u << 9)) >> 6); }
/* normalized-string offset of the shortest key that is a prefix of s[0..n), or -1 */
static long trie_shortest(const orc_t5 *t, const uint8_t *s, size_t n) {
    size_t pos = du_off(t->units[0]);
    for (size_t i = 0; i < n; ++i) {
        const uint8_t c = s[i];
        if (c == 0) return -1;
        pos ^= c;
        if (pos >= t->n_units) return -1;
        const uint32_t u = t->units[pos];
        if ((u & ((1u << 31) | 0xFFu)) != c) return -1;
        pos ^= du_off(u);
        if ((u >> 8) & 1u) return (long)(t->units[pos] & 0x7FFFFFFFu);
    }
    return -1;
}

typedef struct {
    uint8_t *p;
    size_t n, cap;
} bytes_t;
static void bput(bytes_t *b, const void *src, size_t n) {
    if (b->n + n > b->cap) {
        b->cap = (b->n + n) * 2 + 64;
        b->p = (uint8_t *)realloc(b->p, b->cap);
    }
    memcpy(b->p + b->n, src, n);
    b->n += n;
}
static void emit_norm(const orc_t5 *t, long off, bytes_t *o) {
    if ((size_t)off >= t->norm_len) return;
    bput(o, t->norm + off, strlen(t->norm + off));
}

/* Precompiled::normalize of a valid UTF-8 segment. */
static void normalize(const orc_t5 *t, const uint8_t *s, size_t n, bytes_t *o) {
    gstate g;
    orc_gcb_reset(&g);
    size_t i = 0;
    while (i < n) {
        /* cluster [i, j) */
        uint32_t cp;
        size_t j = i + (size_t)u8len(s, n, i, &cp);
        orc_gcb_break(&g, t->prop[cp]);
        while (j < n) {
            int l = u8len(s, n, j, &cp);
            gstate g2 = g;
            if (orc_gcb_break(&g2, t->prop[cp])) break;
            g = g2;
            j += (size_t)l;
        }
        long r = j - i < 6 ? trie_shortest(t, s + i, j - i) : -1;
        if (r >= 0) {
            emit_norm(t, r, o);
        } else {
            for (size_t k = i; k < j;) {
                int l = u8len(s, n, k, &cp);
                long rc = trie_shortest(t, s + k, (size_t)l);
                if (rc >= 0) emit_norm(t, rc, o);
                else bput(o, s + k, (size_t)l);
                k += (size_t)l;
            }
        }
        i = j;
    }
}

/* ---- Unigram ---------------------------------------------------------------- */
typedef struct {
    double score;
    long start; /* -1: unset */
    int id;
} vnode;

static void unigram(const orc_t5 *t, const uint8_t *s, size_t n, idvec *out) {
    if (n == 0) return;
    vnode *best = (vnode *)malloc((n + 1) * sizeof(vnode));
    for (size_t i = 0; i <= n; ++i) { best[i].score = 0.0; best[i].start = -1; best[i].id = -1; }
    for (size_t st = 0; st < n;) {
        uint32_t cp;
        const size_t mb = (size_t)u8len(s, n, st, &cp);
        const double base = best[st].score;
        int single = 0;
        for (size_t e = st + 1; e <= n && (int)(e - st) <= t->max_piece; ++e) {
            int id = vmap_get(&t->vocab, s + st, e - st);
            if (id < 0) continue;
            const double cand = t->score[id] + base;
            if (best[e].start < 0 || cand > best[e].score) {
                best[e].score = cand;
                best[e].start = (long)st;
                best[e].id = id;
            }
            if (e - st == mb) single = 1;
        }
        if (!single) {
            const double cand = t->unk_score + base;
            if (best[st + mb].start < 0 || cand > best[st + mb].score) {
                best[st + mb].score = cand;
                best[st + mb].start = (long)st;
                best[st + mb].id = t->unk_id;
            }
        }
        st += mb;
    }
    /* backtrack, fusing consecutive unk nodes */
    size_t cap = 16, k = 0;
    size_t *seg = (size_t *)malloc(2 * cap * sizeof(size_t)); /* (start, end) pairs, reversed */
    int *unkf = (int *)malloc(cap * sizeof(int));
    for (size_t e = n; e > 0;) {
        const size_t st = (size_t)best[e].start;
        const int is_unk = best[e].id == t->unk_id;
        if (is_unk && k && unkf[k - 1]) {
            seg[2 * (k - 1)] = st; /* extend the fused run leftwards */
        } else {
            if (k == cap) {
                cap *= 2;
                seg = (size_t *)realloc(seg, 2 * cap * sizeof(size_t));
                unkf = (int *)realloc(unkf, cap * sizeof(int));
            }
            seg[2 * k] = st;
            seg[2 * k + 1] = e;
            unkf[k] = is_unk;
            ++k;
        }
        e = st;
    }
    for (size_t q = k; q-- > 0;) {
        const size_t a = seg[2 * q], b = seg[2 * q + 1];
        int id = vmap_get(&t->vocab, s + a, b - a);
        idpush(out, (uint32_t)(id >= 0 ? id : t->unk_id));
    }
    free(seg);
    free(unkf);
    free(best);
}

static const uint8_t META[3] = {0xE2, 0x96, 0x81}; /* U+2581 */

/* WhitespaceSplit + Metaspace + Unigram over a normalized segment. */
static void pretok_unigram(const orc_t5 *t, const uint8_t *s, size_t n, idvec *out) {
    bytes_t w = {0};
    size_t i = 0;
    while (i < n) {
        uint32_t cp;
        int l = u8len(s, n, i, &cp);
        if (t->prop[cp] & P_WS) { i += (size_t)l; continue; }
        size_t j = i;
        while (j < n) {
            int lj = u8len(s, n, j, &cp);
            if (t->prop[cp] & P_WS) break;
            j += (size_t)lj;
        }
        /* word [i, j): Metaspace */
        w.n = 0;
        if (!(j - i >= 3 && !memcmp(s + i, META, 3))) bput(&w, META, 3);
        bput(&w, s + i, j - i);
        size_t a = 0;
        for (size_t q = 3; q + 3 <= w.n; ++q) {
            if (!memcmp(w.p + q, META, 3)) {
                unigram(t, w.p + a, q - a, out);
                a = q;
            }
        }
        unigram(t, w.p + a, w.n - a, out);
        i = j;
    }
    free(w.p);
}

static void encode_segment(const orc_t5 *t, const uint8_t *s, size_t n, idvec *out) {
    if (n == 0) return;
    bytes_t o = {0};
    normalize(t, s, n, &o);
    pretok_unigram(t, o.p, o.n, out);
    free(o.p);
}

/* Tokenizer::encode(text, true).get_ids(): added-token split, segments, "$A </s>". */
void orc_t5_encode_vec(const orc_t5 *t, const uint8_t *raw, size_t rn, idvec *out) {
    size_t n;
    uint8_t *s = sanitize(raw, rn, &n);
    size_t seg = 0, i = 0;
    while (i < n) {
        int best = -1;
        size_t best_len = 0;
        for (int k = 0; k < t->n_special; ++k) {
            const size_t l = t->special_len[k];
            if (l > best_len && i + l <= n && s[i] == (uint8_t)t->special[k][0] && !memcmp(s + i, t->special[k], l)) {
                best = k;
                best_len = l;
            }
        }
        if (best >= 0) {
            encode_segment(t, s + seg, i - seg, out);
            idpush(out, (uint32_t)t->special_id[best]);
            i += best_len;
            seg = i;
        } else {
            ++i;
        }
    }
    encode_segment(t, s + seg, n - seg, out);
    idpush(out, (uint32_t)t->eos_id);
    free(s);
}

long orc_t5_encode(const orc_t5 *t, const uint8_t *s, size_t n, uint32_t *out, size_t cap) {
    idvec v = {0};
    orc_t5_encode_vec(t, s, n, &v);
    size_t m = v.n < cap ? v.n : cap;
    if (out && m) memcpy(out, v.p, m * sizeof(uint32_t));
    free(v.p);
    return (long)v.n;
}

/* Precompiled normalizer alone (for tests): writes at most cap bytes, returns the length. */
long orc_t5_normalize(const orc_t5 *t, const uint8_t *s, size_t n, uint8_t *out, size_t cap) {
    bytes_t o = {0};
    normalize(t, s, n, &o);
    size_t m = o.n < cap ? o.n : cap;
    if (out && m) memcpy(out, o.p, m);
    free(o.p);
    return (long)o.n;
}

/* Cluster boundaries of a valid UTF-8 string (tests): writes the byte offset
 * of every cluster start, returns their count. */
long orc_t5_graphemes(const orc_t5 *t, const uint8_t *s, size_t n, uint32_t *starts, size_t cap) {
    gstate g;
    orc_gcb_reset(&g);
    long k = 0;
    for (size_t i = 0; i < n;) {
        uint32_t cp;
        int l = u8len(s, n, i, &cp);
        if (l == 0) { cp = 0xFFFD; l = 1; }
        if (orc_gcb_break(&g, t->prop[cp]) || i == 0) {
            if ((size_t)k < cap) starts[k] = (uint32_t)i;
            ++k;
        }
        i += (size_t)l;
    }
    return k;
}

/* Framing of TokenizerWrapper::encode_mask for T5 (tokenizer_wrapper.rs:125-131). */
static void t5_encode_cb(const void *impl, const uint8_t *s, size_t n, idvec *out) {
    orc_t5_encode_vec((const orc_t5 *)impl, s, n, out);
}
void orc_encoder_t5(const orc_t5 *t, orc_encoder *e) {
    memset(e, 0, sizeof(*e));
    e->encode = t5_encode_cb;
    e->impl = t;
    e->npre = 1;
    e->pre[0] = (uint32_t)t->eos_id;
    e->npost = 1;
    e->post[0] = (uint32_t)t->eos_id;
    for (int k = 0; k < 100; ++k) {
        char name[32];
        snprintf(name, sizeof(name), "<extra_id_%d>", k);
        e->extra[k] = orc_t5_special_id(t, name);
    }
}
