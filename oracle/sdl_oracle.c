/*
 * sdl_oracle.c -- CPU restatement (plain C) of the reference Batcher hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see sdl_oracle.h).  Straight-line, one record at a
 * time, written for obviousness, not speed.  Each function cites what it
 * restates.  Parity of this file is pinned by tests/test_oracle_golden.py
 * against token ids produced by HF `tokenizers` 0.22.2 (same project as the
 * crate `tokenizers` 0.13.1 the reference pins in rust/Cargo.lock) and against
 * masking fixtures produced by tests/golden/make_goldens.py.
 */
#include "orc_internal.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* Unicode table (tools/make_unicode_tables.py)                               */
/* ------------------------------------------------------------------------- */
enum { C_OTHER = 0, C_WS = 1, C_ISO = 2, C_DEL = 3 };

typedef struct {
    uint32_t n_pages, n_blocks, pool_bytes;
    uint16_t *page;
    uint32_t *entry;
    uint8_t *pool;
} utab;

static int utab_load(utab *u, const char *path) {
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    char magic[4];
    uint32_t hdr[4];
    if (fread(magic, 1, 4, f) != 4 || memcmp(magic, "SDLU", 4) || fread(hdr, 4, 4, f) != 4 || hdr[0] != 2) {
        fclose(f);
        return -1;
    }
    u->n_pages = hdr[1];
    u->n_blocks = hdr[2];
    u->pool_bytes = hdr[3];
    u->page = (uint16_t *)malloc(2 * (size_t)u->n_pages);
    u->entry = (uint32_t *)malloc(4 * 128 * (size_t)u->n_blocks);
    u->pool = (uint8_t *)malloc(u->pool_bytes + 1);
    int ok = fread(u->page, 2, u->n_pages, f) == u->n_pages &&
             fread(u->entry, 4, 128 * (size_t)u->n_blocks, f) == 128 * (size_t)u->n_blocks &&
             fread(u->pool, 1, u->pool_bytes, f) == u->pool_bytes;
    fclose(f);
    return ok ? 0 : -1;
}

static uint32_t utab_get(const utab *u, uint32_t cp) {
    if (cp >= 0x110000u) return C_DEL;
    return u->entry[(size_t)u->page[cp >> 7] * 128 + (cp & 127)];
}

/* UTF-8 decode of one char at s[i] (i < n).  Rust `String` input is always
 * valid UTF-8; anything else decodes to U+FFFD (class DEL, 1 byte). */
static int utf8_decode(const uint8_t *s, size_t n, size_t i, uint32_t *cp) {
    uint8_t b = s[i];
    int len;
    uint32_t c;
    if (b < 0x80) { *cp = b; return 1; }
    if ((b & 0xE0) == 0xC0) { len = 2; c = b & 0x1F; }
    else if ((b & 0xF0) == 0xE0) { len = 3; c = b & 0x0F; }
    else if ((b & 0xF8) == 0xF0) { len = 4; c = b & 0x07; }
    else { *cp = 0xFFFD; return 1; }
    if (i + (size_t)len > n) { *cp = 0xFFFD; return 1; }
    for (int k = 1; k < len; ++k) {
        if ((s[i + k] & 0xC0) != 0x80) { *cp = 0xFFFD; return 1; }
        c = (c << 6) | (s[i + k] & 0x3F);
    }
    *cp = c;
    return len;
}

/* ------------------------------------------------------------------------- */
/* Vocabulary: string -> id (WordPiece model vocab, bert vocab.txt layout)    */
/* ------------------------------------------------------------------------- */
typedef struct {
    char **str;
    int *len;
    int n;
    int *slot; /* open addressing, -1 empty */
    uint32_t mask;
} vocab_t;

static uint64_t fnv(const uint8_t *p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}

static int vocab_find(const vocab_t *v, const uint8_t *p, size_t n) {
    uint32_t i = (uint32_t)fnv(p, n) & v->mask;
    for (;;) {
        int id = v->slot[i];
        if (id < 0) return -1;
        if ((size_t)v->len[id] == n && memcmp(v->str[id], p, n) == 0) return id;
        i = (i + 1) & v->mask;
    }
}

static int vocab_load(vocab_t *v, const char *path) {
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *buf = (char *)malloc((size_t)sz + 1);
    if (fread(buf, 1, (size_t)sz, f) != (size_t)sz) { fclose(f); return -1; }
    fclose(f);
    buf[sz] = 0;
    int cap = 1024;
    v->str = (char **)malloc(sizeof(char *) * cap);
    v->len = (int *)malloc(sizeof(int) * cap);
    v->n = 0;
    char *p = buf;
    while (p < buf + sz) {
        char *e = strchr(p, '\n');
        if (!e) e = buf + sz;
        int l = (int)(e - p);
        if (l > 0 && p[l - 1] == '\r') --l;
        if (v->n == cap) {
            cap *= 2;
            v->str = (char **)realloc(v->str, sizeof(char *) * cap);
            v->len = (int *)realloc(v->len, sizeof(int) * cap);
        }
        v->str[v->n] = p;
        v->len[v->n] = l;
        v->n++;
        p = e + 1;
    }
    uint32_t slots = 1;
    while (slots < (uint32_t)v->n * 2) slots <<= 1;
    v->mask = slots - 1;
    v->slot = (int *)malloc(sizeof(int) * slots);
    for (uint32_t i = 0; i < slots; ++i) v->slot[i] = -1;
    for (int id = 0; id < v->n; ++id) {
        /* HF builds a HashMap from vocab.txt; a duplicated line keeps the last id */
        uint32_t i = (uint32_t)fnv((const uint8_t *)v->str[id], (size_t)v->len[id]) & v->mask;
        for (;;) {
            int o = v->slot[i];
            if (o < 0) { v->slot[i] = id; break; }
            if (v->len[o] == v->len[id] && memcmp(v->str[o], v->str[id], (size_t)v->len[id]) == 0) {
                v->slot[i] = id;
                break;
            }
            i = (i + 1) & v->mask;
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------- */
/* Tokenizer                                                                  */
/* ------------------------------------------------------------------------- */
#define MAX_INPUT_CHARS_PER_WORD 100 /* WordPiece default (tokenizer.json) */
#define N_SPECIAL 5

struct orc_tok {
    vocab_t v;
    utab u;
    int unk, cls, sep;
    const char *special[N_SPECIAL];
    int special_id[N_SPECIAL];
};

orc_tok *orc_tok_load(const char *vocab_txt, const char *unicode_bin) {
    orc_tok *t = (orc_tok *)calloc(1, sizeof(orc_tok));
    if (vocab_load(&t->v, vocab_txt) || utab_load(&t->u, unicode_bin)) {
        free(t);
        return NULL;
    }
    /* bert-base-uncased added tokens: all "normalized": false, so they are
     * matched on the raw text before normalization (AddedVocabulary). */
    static const char *sp[N_SPECIAL] = {"[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"};
    for (int i = 0; i < N_SPECIAL; ++i) {
        t->special[i] = sp[i];
        t->special_id[i] = vocab_find(&t->v, (const uint8_t *)sp[i], strlen(sp[i]));
        if (t->special_id[i] < 0) { free(t); return NULL; }
    }
    t->unk = t->special_id[1];
    t->cls = t->special_id[2];
    t->sep = t->special_id[3];
    return t;
}

void orc_tok_free(orc_tok *t) { free(t); }
int orc_tok_vocab_size(const orc_tok *t) { return t->v.n; }


/* WordPiece::tokenize (tokenizers/src/models/wordpiece/mod.rs): greedy
 * longest-match-first; "##" prefix after the first piece; the whole word is
 * [UNK] if any position cannot be matched or it has > 100 chars. */
static void wordpiece(const orc_tok *t, const uint8_t *w, size_t L, size_t nchars, idvec *out) {
    if (L == 0) return;
    if (nchars > MAX_INPUT_CHARS_PER_WORD) { idpush(out, (uint32_t)t->unk); return; }
    uint8_t buf[4096 + 2];
    size_t mark = out->n;
    size_t start = 0;
    while (start < L) {
        size_t end = L;
        int id = -1;
        while (start < end) {
            size_t k = 0;
            if (start > 0) { buf[0] = '#'; buf[1] = '#'; k = 2; }
            memcpy(buf + k, w + start, end - start);
            id = vocab_find(&t->v, buf, k + end - start);
            if (id >= 0) break;
            /* end -= len_utf8(last char of substr) */
            do { --end; } while (end > start && (w[end] & 0xC0) == 0x80);
        }
        if (id < 0) {
            out->n = mark;
            idpush(out, (uint32_t)t->unk);
            return;
        }
        idpush(out, (uint32_t)id);
        start = end;
    }
}

/* NFD canonical ordering of the combining marks strip_accents keeps
 * (unicode-normalization's decompose + stable sort by ccc, then the Mn filter):
 * kept marks (table bit 4 + ccc) wait in a run, which ends -- sorted, stable --
 * at any char holding a starter (bit 4 on a DEL char: a removed starter). */
typedef struct {
    uint8_t bytes[64][4];
    uint8_t len[64], ccc[64];
    int n;
} mark_run;

static void run_flush(mark_run *r, uint8_t *word, size_t *wl, size_t cap, int *overflow) {
    for (int pass = 1; pass < r->n; ++pass)  /* insertion sort: stable */
        for (int j = pass; j > 0 && r->ccc[j - 1] > r->ccc[j]; --j) {
            uint8_t tb[4], tl = r->len[j], tc = r->ccc[j];
            memcpy(tb, r->bytes[j], 4);
            memcpy(r->bytes[j], r->bytes[j - 1], 4);
            r->len[j] = r->len[j - 1];
            r->ccc[j] = r->ccc[j - 1];
            memcpy(r->bytes[j - 1], tb, 4);
            r->len[j - 1] = tl;
            r->ccc[j - 1] = tc;
        }
    for (int k = 0; k < r->n; ++k) {
        if (*wl + r->len[k] > cap) *overflow = 1;
        else { memcpy(word + *wl, r->bytes[k], r->len[k]); *wl += r->len[k]; }
    }
    r->n = 0;
}

static void run_push(mark_run *r, const uint8_t *b, int len, int ccc, uint8_t *word, size_t *wl, size_t cap,
                     int *overflow) {
    if (r->n == 64) run_flush(r, word, wl, cap, overflow); /* > 64 marks in a row: the word is [UNK] anyway */
    memcpy(r->bytes[r->n], b, (size_t)len);
    r->len[r->n] = (uint8_t)len;
    r->ccc[r->n] = (uint8_t)ccc;
    r->n++;
}

/* BertNormalizer + BertPreTokenizer over one non-special segment, feeding each
 * word to WordPiece.  Per-char behaviour comes from the probed table. */
static void encode_segment(const orc_tok *t, const uint8_t *s, size_t n, idvec *out) {
    uint8_t word[4096];
    size_t wl = 0, wc = 0;
    int overflow = 0;
    mark_run run;
    run.n = 0;
    size_t i = 0;
    while (i < n) {
        uint32_t cp;
        int len = utf8_decode(s, n, i, &cp);
        uint32_t e = utab_get(&t->u, cp);
        uint32_t cls = e & 3;
        const uint8_t *mb = s + i;
        size_t ml = (size_t)len, mc = 1;
        if (!(e & 4) && cls != C_DEL && cls != C_WS) {
            const uint8_t *pe = t->u.pool + (e >> 8);
            ml = pe[0];
            mc = pe[1];
            mb = pe + 2;
        }
        i += (size_t)len;
        if (cls == C_DEL) {
            if (e & 16) run_flush(&run, word, &wl, sizeof(word), &overflow); /* a removed starter */
            continue;
        }
        if (cls == C_WS || cls == C_ISO) {
            run_flush(&run, word, &wl, sizeof(word), &overflow);
            if (wl || overflow) {
                if (overflow) idpush(out, (uint32_t)t->unk);
                else wordpiece(t, word, wl, wc, out);
            }
            wl = wc = 0;
            overflow = 0;
            if (cls == C_ISO) wordpiece(t, mb, ml, mc, out);
            continue;
        }
        /* OTHER: extend the current word */
        wc += mc;
        if (e & 16) {
            if (e & 4) { /* a kept mark */
                run_push(&run, mb, (int)ml, (int)((e >> 8) & 0xFF), word, &wl, sizeof(word), &overflow);
                continue;
            }
            /* precomposed: its starters end the run, its kept marks join it */
            for (size_t q = 0; q < ml;) {
                uint32_t c2;
                int l2 = utf8_decode(mb, ml, q, &c2);
                uint32_t e2 = utab_get(&t->u, c2);
                if ((e2 & 16) && (e2 & 4) && (e2 & 3) == C_OTHER) {
                    run_push(&run, mb + q, l2, (int)((e2 >> 8) & 0xFF), word, &wl, sizeof(word), &overflow);
                } else {
                    run_flush(&run, word, &wl, sizeof(word), &overflow);
                    if (wl + (size_t)l2 > sizeof(word)) overflow = 1;
                    else { memcpy(word + wl, mb + q, (size_t)l2); wl += (size_t)l2; }
                }
                q += (size_t)l2;
            }
            continue;
        }
        run_flush(&run, word, &wl, sizeof(word), &overflow);
        if (wl + ml > sizeof(word)) overflow = 1; /* > 100 chars for sure */
        else { memcpy(word + wl, mb, ml); wl += ml; }
    }
    run_flush(&run, word, &wl, sizeof(word), &overflow);
    if (overflow) idpush(out, (uint32_t)t->unk);
    else if (wl) wordpiece(t, word, wl, wc, out);
}

/* Tokenizer::encode(text, true): AddedVocabulary split (leftmost-longest match
 * of the special strings on the raw text), each remaining segment normalized +
 * pre-tokenized + WordPiece, then TemplateProcessing "[CLS] $A [SEP]". */
void orc_bert_encode_vec(const orc_tok *t, const uint8_t *s, size_t n, idvec *out) {
    idpush(out, (uint32_t)t->cls);
    size_t seg = 0, i = 0;
    while (i < n) {
        int best = -1;
        size_t best_len = 0;
        if (s[i] == '[') {
            for (int k = 0; k < N_SPECIAL; ++k) {
                size_t l = strlen(t->special[k]);
                if (i + l <= n && memcmp(s + i, t->special[k], l) == 0 && l > best_len) {
                    best = k;
                    best_len = l;
                }
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
    idpush(out, (uint32_t)t->sep);
}

long orc_bert_encode(const orc_tok *t, const uint8_t *s, size_t n, uint32_t *out, size_t cap) {
    idvec v = {0};
    orc_bert_encode_vec(t, s, n, &v);
    size_t m = v.n < cap ? v.n : cap;
    if (out && m) memcpy(out, v.p, m * sizeof(uint32_t));
    free(v.p);
    return (long)v.n;
}

/* Framing of TokenizerWrapper::encode_mask for BERT (tokenizer_wrapper.rs:107-116):
 * [CLS] + encode(text, true) + [SEP] [SEP]. */
static void bert_encode_cb(const void *impl, const uint8_t *s, size_t n, idvec *out) {
    orc_bert_encode_vec((const orc_tok *)impl, s, n, out);
}

void orc_encoder_bert(const orc_tok *t, orc_encoder *e) {
    memset(e, 0, sizeof(*e));
    e->encode = bert_encode_cb;
    e->impl = t;
    e->npre = 1;
    e->pre[0] = (uint32_t)t->cls;
    e->npost = 2;
    e->post[0] = (uint32_t)t->sep;
    e->post[1] = (uint32_t)t->sep;
}
