/*
 * orc_bpe.c -- CPU restatement of the gpt2 tokenizer (TEST INFRASTRUCTURE ONLY).
 *
 * What the reference calls for task=clm: TokenizerHolder::get_ids ->
 * tokenizers::Tokenizer::encode(text, true) (rust/src/tokenizer/tokenizer_holder.rs:19-28,
 * crate tokenizers 0.13.1, not vendored) with the hub's gpt2 tokenizer.json:
 *   AddedVocabulary split (<|endoftext|>, leftmost-longest on the raw text)
 *   -> ByteLevel pre-tokenizer: the GPT-2 regex
 *        's|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+
 *      (pre_tokenizers/byte_level.rs), applied here as a literal left-to-right
 *      scan trying the alternatives in order, with per-code-point classes
 *      probed from the tokenizers binding (data/gpt2_classes.bin);
 *   -> BPE per pre-token on its bytes' byte-level symbols: tokenizers'
 *      Word::merge_all (models/bpe/word.rs) -- a min-heap of (rank, position),
 *      stale entries skipped;
 *   -> ByteLevel post-processor (adds no ids).
 * Then TokenizerWrapper::encode_mask framing for Gpt: [eos] + ids + [eos]
 * (tokenizer_wrapper.rs:118-124).
 *
 * Input bytes that are not valid UTF-8 cannot reach the reference (a Rust
 * String); here every char is either a complete lead + continuation sequence
 * (overlong forms decoded as is) or a single byte of class O.
 */
#include <stdio.h>
#include <string.h>

#include "orc_internal.h"
#include "orc_json.h"

enum { GO = 0, GL = 1, GN = 2, GW = 3 };

typedef struct {
    char **keys;
    size_t *lens;
    int *vals;
    size_t cap;
} smap;

static uint64_t sh(const char *p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ (uint8_t)p[i]) * 1099511628211ull;
    return h;
}
static void smap_init(smap *m, size_t n) {
    m->cap = 16;
    while (m->cap < 2 * n + 16) m->cap <<= 1;
    m->keys = (char **)calloc(m->cap, sizeof(char *));
    m->lens = (size_t *)calloc(m->cap, sizeof(size_t));
    m->vals = (int *)calloc(m->cap, sizeof(int));
}
static int smap_get(const smap *m, const char *k, size_t n) {
    for (size_t i = sh(k, n) & (m->cap - 1);; i = (i + 1) & (m->cap - 1)) {
        if (!m->keys[i]) return -1;
        if (m->lens[i] == n && !memcmp(m->keys[i], k, n)) return m->vals[i];
    }
}
static void smap_put(smap *m, const char *k, size_t n, int v) {
    for (size_t i = sh(k, n) & (m->cap - 1);; i = (i + 1) & (m->cap - 1)) {
        if (!m->keys[i]) {
            m->keys[i] = (char *)malloc(n + 1);
            memcpy(m->keys[i], k, n);
            m->keys[i][n] = 0;
            m->lens[i] = n;
            m->vals[i] = v;
            return;
        }
        if (m->lens[i] == n && !memcmp(m->keys[i], k, n)) { m->vals[i] = v; return; }
    }
}
static void smap_free(smap *m) {
    for (size_t i = 0; i < m->cap; ++i) free(m->keys[i]);
    free(m->keys);
    free(m->lens);
    free(m->vals);
}

typedef struct { uint32_t key, rank, id; } ment;

struct orc_gpt2 {
    smap vocab;
    int byte_id[256];
    ment *merges; /* open addressing on key = a << 16 | b */
    size_t mcap;
    uint8_t *cls;  /* 0x110000 classes */
    char *added[8];
    size_t added_len[8];
    int added_id[8];
    int n_added;
    int eos;
};

static void madd(orc_gpt2 *t, uint32_t key, uint32_t rank, uint32_t id) {
    for (size_t i = (key * 2654435761u) & (t->mcap - 1);; i = (i + 1) & (t->mcap - 1)) {
        if (t->merges[i].key == 0xFFFFFFFFu) { t->merges[i] = (ment){key, rank, id}; return; }
        if (t->merges[i].key == key) return; /* first rank wins */
    }
}
static const ment *mget(const orc_gpt2 *t, uint32_t a, uint32_t b) {
    const uint32_t key = a << 16 | b;
    for (size_t i = (key * 2654435761u) & (t->mcap - 1);; i = (i + 1) & (t->mcap - 1)) {
        if (t->merges[i].key == 0xFFFFFFFFu) return NULL;
        if (t->merges[i].key == key) return &t->merges[i];
    }
}

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

/* GPT-2 bytes_to_unicode() */
static void byte_cps(uint32_t cp[256]) {
    uint32_t n = 0;
    for (uint32_t b = 0; b < 256; ++b) {
        int direct = (b >= '!' && b <= '~') || (b >= 0xA1 && b <= 0xAC) || (b >= 0xAE);
        cp[b] = direct ? b : 256 + n++;
    }
}
static size_t utf8(char *o, uint32_t c) {
    if (c < 0x80) { o[0] = (char)c; return 1; }
    o[0] = (char)(0xC0 | (c >> 6));
    o[1] = (char)(0x80 | (c & 63));
    return 2; /* stand-ins are < 0x800 */
}

static int load_classes(orc_gpt2 *t, const char *path) {
    size_t n;
    char *b = slurp(path, &n);
    if (!b || n < 16 || memcmp(b, "SDLG", 4)) { free(b); return -1; }
    uint32_t np, nb;
    memcpy(&np, b + 8, 4);
    memcpy(&nb, b + 12, 4);
    if (np != 0x110000 / 256 || n != 16 + 2 * (size_t)np + 64 * (size_t)nb) { free(b); return -1; }
    t->cls = (uint8_t *)malloc(0x110000);
    const uint16_t *page = (const uint16_t *)(b + 16);
    const uint8_t *blk = (const uint8_t *)(b + 16 + 2 * np);
    for (uint32_t cp = 0; cp < 0x110000; ++cp)
        t->cls[cp] = (blk[(size_t)page[cp >> 8] * 64 + ((cp & 255) >> 2)] >> (2 * (cp & 3))) & 3;
    free(b);
    return 0;
}

orc_gpt2 *orc_gpt2_load(const char *tokenizer_json, const char *classes_bin) {
    size_t n;
    char *body = slurp(tokenizer_json, &n);
    if (!body) return NULL;
    oj *root = oj_parse(body, n);
    free(body);
    if (!root) return NULL;
    orc_gpt2 *t = (orc_gpt2 *)calloc(1, sizeof(orc_gpt2));
    const oj *model = oj_get(root, "model");
    const oj *vocab = oj_get(model, "vocab"), *merges = oj_get(model, "merges");
    if (!vocab || !merges || load_classes(t, classes_bin)) goto fail;
    smap_init(&t->vocab, vocab->n + 16);
    for (size_t i = 0; i < vocab->n; ++i) smap_put(&t->vocab, vocab->keys[i], vocab->klens[i], (int)vocab->items[i].num);
    uint32_t cp[256];
    byte_cps(cp);
    for (int b = 0; b < 256; ++b) {
        char u[4];
        size_t l = utf8(u, cp[b]);
        t->byte_id[b] = smap_get(&t->vocab, u, l);
        if (t->byte_id[b] < 0) goto fail;
    }
    t->mcap = 16;
    while (t->mcap < 2 * merges->n + 16) t->mcap <<= 1;
    t->merges = (ment *)malloc(t->mcap * sizeof(ment));
    memset(t->merges, 0xFF, t->mcap * sizeof(ment));
    for (size_t r = 0; r < merges->n; ++r) {
        const oj *m = &merges->items[r];
        const char *a, *b;
        size_t la, lb;
        if (m->kind == OJ_STR) {
            const char *sp = memchr(m->str + 1, ' ', m->slen - 1);
            if (!sp) goto fail;
            a = m->str;
            la = (size_t)(sp - m->str);
            b = sp + 1;
            lb = m->slen - la - 1;
        } else if (m->kind == OJ_ARR && m->n == 2) {
            a = m->items[0].str;
            la = m->items[0].slen;
            b = m->items[1].str;
            lb = m->items[1].slen;
        } else {
            goto fail;
        }
        char *ab = (char *)malloc(la + lb + 1);
        memcpy(ab, a, la);
        memcpy(ab + la, b, lb);
        int ia = smap_get(&t->vocab, a, la), ib = smap_get(&t->vocab, b, lb), ic = smap_get(&t->vocab, ab, la + lb);
        free(ab);
        if (ia < 0 || ib < 0 || ic < 0) goto fail;
        madd(t, (uint32_t)ia << 16 | (uint32_t)ib, (uint32_t)r, (uint32_t)ic);
    }
    const oj *added = oj_get(root, "added_tokens");
    t->eos = -1;
    for (size_t i = 0; added && i < added->n && t->n_added < 8; ++i) {
        const oj *c = oj_get(&added->items[i], "content"), *id = oj_get(&added->items[i], "id");
        if (!c || !id) continue;
        t->added[t->n_added] = (char *)malloc(c->slen + 1);
        memcpy(t->added[t->n_added], c->str, c->slen + 1);
        t->added_len[t->n_added] = c->slen;
        t->added_id[t->n_added] = (int)id->num;
        if (!strcmp(c->str, "<|endoftext|>")) t->eos = (int)id->num;
        t->n_added++;
    }
    oj_free(root);
    if (t->eos < 0) { orc_gpt2_free(t); return NULL; }
    return t;
fail:
    oj_free(root);
    orc_gpt2_free(t);
    return NULL;
}

void orc_gpt2_free(orc_gpt2 *t) {
    if (!t) return;
    if (t->vocab.keys) smap_free(&t->vocab);
    free(t->merges);
    free(t->cls);
    for (int i = 0; i < t->n_added; ++i) free(t->added[i]);
    free(t);
}

/* ---- BPE: Word::merge_all with a binary min-heap of (rank, pos) ------------ */
typedef struct { uint32_t rank, pos, id; } hent;
static int hless(const hent *a, const hent *b) { return a->rank != b->rank ? a->rank < b->rank : a->pos < b->pos; }

static void bpe_word(const orc_gpt2 *t, const uint8_t *s, size_t n, idvec *out) {
    if (n == 0) return;
    int *id = (int *)malloc(n * sizeof(int)), *prv = (int *)malloc(n * sizeof(int)), *nxt = (int *)malloc(n * sizeof(int));
    char *live = (char *)malloc(n);
    size_t hcap = 4 * n + 4, hn = 0;
    hent *h = (hent *)malloc(hcap * sizeof(hent));
    for (size_t i = 0; i < n; ++i) {
        id[i] = t->byte_id[s[i]];
        prv[i] = (int)i - 1;
        nxt[i] = i + 1 < n ? (int)i + 1 : -1;
        live[i] = 1;
    }
#define HPUSH(E)                                                                  \
    do {                                                                          \
        if (hn == hcap) { hcap *= 2; h = (hent *)realloc(h, hcap * sizeof(hent)); } \
        size_t k_ = hn++;                                                         \
        h[k_] = (E);                                                              \
        while (k_ && hless(&h[k_], &h[(k_ - 1) / 2])) {                           \
            hent tmp_ = h[k_]; h[k_] = h[(k_ - 1) / 2]; h[(k_ - 1) / 2] = tmp_;   \
            k_ = (k_ - 1) / 2;                                                    \
        }                                                                         \
    } while (0)
    for (size_t i = 0; i + 1 < n; ++i) {
        const ment *m = mget(t, (uint32_t)id[i], (uint32_t)id[i + 1]);
        if (m) HPUSH(((hent){m->rank, (uint32_t)i, m->id}));
    }
    while (hn) {
        hent top = h[0];
        h[0] = h[--hn];
        for (size_t k = 0;;) { /* sift down */
            size_t l = 2 * k + 1, r = l + 1, b = k;
            if (l < hn && hless(&h[l], &h[b])) b = l;
            if (r < hn && hless(&h[r], &h[b])) b = r;
            if (b == k) break;
            hent tmp = h[k]; h[k] = h[b]; h[b] = tmp;
            k = b;
        }
        const int pos = (int)top.pos;
        if (!live[pos] || nxt[pos] < 0) continue;
        const int nx = nxt[pos];
        const ment *m = mget(t, (uint32_t)id[pos], (uint32_t)id[nx]);
        if (!m || m->id != top.id) continue; /* expired */
        id[pos] = (int)top.id;
        live[nx] = 0;
        nxt[pos] = nxt[nx];
        if (nxt[pos] >= 0) prv[nxt[pos]] = pos;
        if (prv[pos] >= 0) {
            const ment *a = mget(t, (uint32_t)id[prv[pos]], (uint32_t)id[pos]);
            if (a) HPUSH(((hent){a->rank, (uint32_t)prv[pos], a->id}));
        }
        if (nxt[pos] >= 0) {
            const ment *b = mget(t, (uint32_t)id[pos], (uint32_t)id[nxt[pos]]);
            if (b) HPUSH(((hent){b->rank, (uint32_t)pos, b->id}));
        }
    }
#undef HPUSH
    for (size_t i = 0; i < n; ++i)
        if (live[i]) idpush(out, (uint32_t)id[i]);
    free(id); free(prv); free(nxt); free(live); free(h);
}

/* ---- ByteLevel pre-tokenizer: the GPT-2 regex as a literal scan ----------- */
typedef struct { size_t start, len; int cls; } gch;

static int cls_of(const orc_gpt2 *t, const uint8_t *s, size_t n, size_t i, size_t *len) {
    const uint8_t b = s[i];
    *len = 1;
    if (b < 0x80) return t->cls[b];
    int need;
    uint32_t cp;
    if ((b & 0xE0) == 0xC0) { need = 2; cp = b & 0x1F; }
    else if ((b & 0xF0) == 0xE0) { need = 3; cp = b & 0x0F; }
    else if ((b & 0xF8) == 0xF0) { need = 4; cp = b & 0x07; }
    else return GO; /* continuation byte or invalid lead: one O byte */
    if (i + (size_t)need > n) return GO;
    for (int j = 1; j < need; ++j) {
        if ((s[i + j] & 0xC0) != 0x80) return GO;
        cp = (cp << 6) | (s[i + j] & 0x3F);
    }
    *len = (size_t)need;
    return cp < 0x110000 ? t->cls[cp] : GO;
}

static void pretok_segment(const orc_gpt2 *t, const uint8_t *s, size_t n, idvec *out) {
    size_t cap = 64, nc = 0;
    gch *c = (gch *)malloc(cap * sizeof(gch));
    for (size_t i = 0; i < n;) {
        size_t len;
        int k = cls_of(t, s, n, i, &len);
        if (nc == cap) { cap *= 2; c = (gch *)realloc(c, cap * sizeof(gch)); }
        c[nc++] = (gch){i, len, k};
        i += len;
    }
#define BYTE(j) (c[j].len == 1 ? (int)s[c[j].start] : -1)
    size_t i = 0;
    while (i < nc) {
        size_t j = i + 1;
        const int b = BYTE(i);
        int done = 0;
        if (b == '\'') { /* 's|'t|'re|'ve|'m|'ll|'d */
            const int b1 = i + 1 < nc ? BYTE(i + 1) : -1, b2 = i + 2 < nc ? BYTE(i + 2) : -1;
            if (b1 == 's' || b1 == 't' || b1 == 'm' || b1 == 'd') { j = i + 2; done = 1; }
            else if ((b1 == 'r' && b2 == 'e') || (b1 == 'v' && b2 == 'e') || (b1 == 'l' && b2 == 'l')) { j = i + 3; done = 1; }
        }
        for (int want = GL; !done && want <= 3; ++want) { /* ` ?\p{L}+`, ` ?\p{N}+`, ` ?[^\s\p{L}\p{N}]+` */
            const int wc = want == 3 ? GO : want;
            size_t a = i;
            if (b == ' ' && i + 1 < nc && c[i + 1].cls == wc) a = i + 1;
            if (c[a].cls != wc) continue;
            j = a;
            while (j < nc && c[j].cls == wc) ++j;
            done = 1;
        }
        if (!done) { /* `\s+(?!\S)` then `\s+` */
            j = i;
            while (j < nc && c[j].cls == GW) ++j;
            if (j < nc && j - i >= 2) --j;
        }
        const size_t a0 = c[i].start, a1 = j < nc ? c[j].start : n;
        bpe_word(t, s + a0, a1 - a0, out);
        i = j;
    }
#undef BYTE
    free(c);
}

void orc_gpt2_encode_vec(const orc_gpt2 *t, const uint8_t *s, size_t n, idvec *out) {
    size_t seg = 0, i = 0;
    while (i < n) { /* AddedVocabulary: leftmost-longest added token */
        int best = -1;
        size_t bl = 0;
        for (int k = 0; k < t->n_added; ++k)
            if (t->added_len[k] > bl && i + t->added_len[k] <= n && !memcmp(s + i, t->added[k], t->added_len[k])) {
                best = k;
                bl = t->added_len[k];
            }
        if (best < 0) { ++i; continue; }
        pretok_segment(t, s + seg, i - seg, out);
        idpush(out, (uint32_t)t->added_id[best]);
        i += bl;
        seg = i;
    }
    pretok_segment(t, s + seg, n - seg, out);
}

long orc_gpt2_encode(const orc_gpt2 *t, const uint8_t *s, size_t n, uint32_t *out, size_t cap) {
    idvec v = {0};
    orc_gpt2_encode_vec(t, s, n, &v);
    size_t m = v.n < cap ? v.n : cap;
    if (out && m) memcpy(out, v.p, m * sizeof(uint32_t));
    free(v.p);
    return (long)v.n;
}

int orc_gpt2_eos(const orc_gpt2 *t) { return t->eos; }

static void gpt2_encode_cb(const void *impl, const uint8_t *s, size_t n, idvec *out) {
    orc_gpt2_encode_vec((const orc_gpt2 *)impl, s, n, out);
}

void orc_encoder_gpt2(const orc_gpt2 *t, orc_encoder *e) {
    memset(e, 0, sizeof(*e));
    e->encode = gpt2_encode_cb;
    e->impl = t;
    e->npre = 1;
    e->pre[0] = (uint32_t)t->eos;
    e->npost = 1;
    e->post[0] = (uint32_t)t->eos;
}
