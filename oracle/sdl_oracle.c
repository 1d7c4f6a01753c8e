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
#include "sdl_oracle.h"

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
    if (fread(magic, 1, 4, f) != 4 || memcmp(magic, "SDLU", 4) || fread(hdr, 4, 4, f) != 4 || hdr[0] != 1) {
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

typedef struct {
    uint32_t *p;
    size_t n, cap;
} idvec;

static void idpush(idvec *v, uint32_t x) {
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 256;
        v->p = (uint32_t *)realloc(v->p, v->cap * sizeof(uint32_t));
    }
    v->p[v->n++] = x;
}

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

/* BertNormalizer + BertPreTokenizer over one non-special segment, feeding each
 * word to WordPiece.  Per-char behaviour comes from the probed table. */
static void encode_segment(const orc_tok *t, const uint8_t *s, size_t n, idvec *out) {
    uint8_t word[4096];
    size_t wl = 0, wc = 0;
    int overflow = 0;
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
        if (cls == C_DEL) continue;
        if (cls == C_WS || cls == C_ISO) {
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
        if (wl + ml > sizeof(word)) overflow = 1; /* > 100 chars for sure */
        else { memcpy(word + wl, mb, ml); wl += ml; }
        wc += mc;
    }
    if (overflow) idpush(out, (uint32_t)t->unk);
    else if (wl) wordpiece(t, word, wl, wc, out);
}

/* Tokenizer::encode(text, true): AddedVocabulary split (leftmost-longest match
 * of the special strings on the raw text), each remaining segment normalized +
 * pre-tokenized + WordPiece, then TemplateProcessing "[CLS] $A [SEP]". */
static void bert_encode_vec(const orc_tok *t, const uint8_t *s, size_t n, idvec *out) {
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
    bert_encode_vec(t, s, n, &v);
    size_t m = v.n < cap ? v.n : cap;
    if (out && m) memcpy(out, v.p, m * sizeof(uint32_t));
    free(v.p);
    return (long)v.n;
}

/* ------------------------------------------------------------------------- */
/* RNG contract: Philox4x32-10 (Salmon et al., SC'11 / Random123)             */
/* ------------------------------------------------------------------------- */
static void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
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
/* Batcher: GenTokenizer(chunk=true) + BertData(Mask)                         */
/* ------------------------------------------------------------------------- */
typedef struct {
    int32_t *d; /* 4 planes of [B,S]: input_ids, attention_mask, token_type_ids, labels */
    int index;
} obatch;

struct orc_batcher {
    const orc_tok *t;
    int task, B, S, mask_length, mask_id;
    uint64_t seed, n_records;
    obatch **q;
    int qh, qn, qcap;
};

/* BertData::new (bert_data.rs:27-38); labels plane starts at -100 */
static obatch *obatch_new(int B, int S) {
    obatch *b = (obatch *)malloc(sizeof(obatch));
    size_t bs = (size_t)B * S;
    b->d = (int32_t *)malloc(4 * bs * sizeof(int32_t));
    for (size_t i = 0; i < bs; ++i) {
        b->d[i] = 0;
        b->d[bs + i] = 1;
        b->d[2 * bs + i] = 0;
        b->d[3 * bs + i] = -100;
    }
    b->index = 0;
    return b;
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

orc_batcher *orc_batcher_new(const orc_tok *t, int task, int batch_size, int seq_len,
                             int mask_length, int mask_id, uint64_t seed) {
    if (task != 0 || batch_size <= 0 || seq_len <= 0 || mask_length < 0 || mask_length > seq_len) return NULL;
    orc_batcher *b = (orc_batcher *)calloc(1, sizeof(orc_batcher));
    b->t = t;
    b->task = task;
    b->B = batch_size;
    b->S = seq_len;
    b->mask_length = mask_length;
    b->mask_id = mask_id;
    b->seed = seed;
    q_push(b, obatch_new(b->B, b->S)); /* GenTokenizer::new (gen_batcher.rs:23-41) */
    return b;
}

typedef struct { uint32_t key, pos; } kp;
static int kp_cmp(const void *a, const void *b) {
    const kp *x = (const kp *)a, *y = (const kp *)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->pos < y->pos ? -1 : (x->pos > y->pos);
}

/* BertData::put_data (bert_data.rs:55-89) with DataSetConfig::Mask, and
 * mask_batch (bert_data.rs:40-53) under the seeded RNG contract. */
static void bert_put_data(orc_batcher *b, obatch *x, const uint32_t *ids, size_t n, uint64_t rec, uint32_t chunk) {
    int S = b->S;
    size_t bs = (size_t)b->B * S;
    int32_t *in = x->d + (size_t)x->index * S;
    int32_t *am = x->d + bs + (size_t)x->index * S;
    int32_t *lb = x->d + 3 * bs + (size_t)x->index * S;
    size_t l = n < (size_t)S ? n : (size_t)S;
    for (size_t j = 0; j < l; ++j) in[j] = (int32_t)ids[j];
    if (n < (size_t)S)
        for (size_t j = (size_t)S - n; j < (size_t)S; ++j) am[j] = 0; /* reversed-range quirk */
    kp *perm = (kp *)malloc(sizeof(kp) * S);
    for (int p = 0; p < S; ++p) {
        perm[p].key = orc_mlm_key(b->seed, rec, chunk, (uint32_t)p);
        perm[p].pos = (uint32_t)p;
    }
    qsort(perm, (size_t)S, sizeof(kp), kp_cmp);
    for (int j = 0; j < S; ++j) lb[j] = -100;
    for (int k = 0; k < b->mask_length; ++k) {
        uint32_t p = perm[k].pos;
        if (in[p] != 0) {
            lb[p] = in[p];
            in[p] = b->mask_id;
        }
    }
    free(perm);
    x->index++;
}

static void batch_out(orc_batcher *b, obatch *x, int32_t *out, int *rows) {
    if (out) memcpy(out, x->d, 4 * (size_t)b->B * b->S * sizeof(int32_t));
    if (rows) *rows = x->index;
    free(x->d);
    free(x);
}

int orc_batcher_push(orc_batcher *b, const uint8_t *s, size_t n, int32_t *out, int *rows) {
    uint64_t rec = b->n_records++;
    /* TokenizerWrapper::encode_mask (tokenizer_wrapper.rs:107-116):
     * [CLS] + encode(text, true) + [SEP] + [SEP] */
    idvec v = {0};
    idpush(&v, (uint32_t)b->t->cls);
    bert_encode_vec(b->t, s, n, &v);
    idpush(&v, (uint32_t)b->t->sep);
    idpush(&v, (uint32_t)b->t->sep);
    if (v.n < 64) { /* gen_batcher.rs:74-76 */
        free(v.p);
        return 0;
    }
    uint32_t chunk = 0;
    for (size_t off = 0; off < v.n; off += (size_t)b->S, ++chunk) { /* chunks_mut(S) */
        size_t len = v.n - off < (size_t)b->S ? v.n - off : (size_t)b->S;
        obatch *back = b->q[b->qh + b->qn - 1];
        bert_put_data(b, back, v.p + off, len, rec, chunk); /* handle_internal_batch */
        if (back->index == b->B) q_push(b, obatch_new(b->B, b->S));
    }
    free(v.p);
    obatch *front = b->q[b->qh];
    if (front->index == b->B) { /* gen_batcher.rs:86-91: at most one batch per call */
        b->qh++;
        b->qn--;
        batch_out(b, front, out, rows);
        return 1;
    }
    return 0;
}

int orc_batcher_flush(orc_batcher *b, int32_t *out, int *rows) {
    if (b->qn == 0) return 0; /* get_working_batch = store.pop_front() */
    obatch *front = b->q[b->qh];
    b->qh++;
    b->qn--;
    batch_out(b, front, out, rows);
    return 1;
}

void orc_batcher_free(orc_batcher *b) {
    for (int i = 0; i < b->qn; ++i) {
        free(b->q[b->qh + i]->d);
        free(b->q[b->qh + i]);
    }
    free(b->q);
    free(b);
}

void orc_batcher_set_next_record(orc_batcher *b, uint64_t record) { b->n_records = record; }
