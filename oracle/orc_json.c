/* orc_json.c -- minimal JSON parser for the CPU oracle (TEST INFRASTRUCTURE ONLY). */
#include "orc_json.h"

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    const char *s;
    size_t n, i;
    int err;
} ps;

static void ws(ps *p) {
    while (p->i < p->n && (p->s[p->i] == ' ' || p->s[p->i] == '\n' || p->s[p->i] == '\r' || p->s[p->i] == '\t')) p->i++;
}

/* A JSON number as serde_json 1.0.87 reads it into an f64 with its default
 * features (rust/Cargo.lock:2037-2040; `float_roundtrip` off), which is how
 * tokenizers' Unigram gets its piece scores (Vec<(String, f64)>):
 * de.rs parse_integer / parse_long_integer / parse_decimal /
 * parse_decimal_overflow / parse_exponent / f64_from_parts.  Digits
 * accumulate in a u64 significand; a digit that would overflow it ends the
 * accumulation (later integer digits only raise the exponent, later fraction
 * digits are dropped); then (double)significand is multiplied or divided by
 * the correctly rounded 10^|e| (e beyond 308 divides by 1e308 first).  Two
 * roundings, so a 17-digit score can land one ulp from strtod's value --
 * which decides Viterbi ties (tests/test_serde_numbers.py pins this against
 * tokenizers itself). */
static double pow10_tab(int k) {
    static double t[309];
    static int init;
    if (!init) {
        char b[16];
        for (int i = 0; i < 309; ++i) {
            snprintf(b, sizeof b, "1e%d", i);
            t[i] = strtod(b, NULL); /* correctly rounded, like Rust's POW10 literals */
        }
        init = 1;
    }
    return t[k];
}

static int isdig(const ps *p) { return p->i < p->n && p->s[p->i] >= '0' && p->s[p->i] <= '9'; }

static int serde_number(ps *p, double *out) {
    const uint64_t M10 = UINT64_MAX / 10, R10 = UINT64_MAX % 10;
    int pos = 1;
    if (p->i < p->n && p->s[p->i] == '-') { pos = 0; p->i++; }
    if (!isdig(p)) return -1;
    uint64_t sig = 0;
    long exp = 0;
    if (p->s[p->i] == '0') {
        p->i++;
        if (isdig(p)) return -1; /* one leading zero only */
    } else {
        while (isdig(p)) {
            const uint64_t d = (uint64_t)(p->s[p->i] - '0');
            if (sig >= M10 && (sig > M10 || d > R10)) { /* parse_long_integer */
                while (isdig(p)) { p->i++; exp++; }
                break;
            }
            sig = sig * 10 + d;
            p->i++;
        }
    }
    if (p->i < p->n && p->s[p->i] == '.') {
        p->i++;
        if (!isdig(p)) return -1;
        while (isdig(p)) {
            const uint64_t d = (uint64_t)(p->s[p->i] - '0');
            if (sig >= M10 && (sig > M10 || d > R10)) { /* parse_decimal_overflow */
                while (isdig(p)) p->i++;
                break;
            }
            sig = sig * 10 + d;
            exp--;
            p->i++;
        }
    }
    if (p->i < p->n && (p->s[p->i] == 'e' || p->s[p->i] == 'E')) {
        p->i++;
        int pe = 1;
        if (p->i < p->n && (p->s[p->i] == '+' || p->s[p->i] == '-')) pe = p->s[p->i++] == '+';
        if (!isdig(p)) return -1;
        long e = 0;
        int ovf = 0;
        while (isdig(p)) {
            const long d = p->s[p->i++] - '0';
            if (e >= INT32_MAX / 10 && (e > INT32_MAX / 10 || d > INT32_MAX % 10)) ovf = 1;
            if (!ovf) e = e * 10 + d;
        }
        if (ovf) { /* parse_exponent_overflow: 0 for a zero significand or a negative exponent */
            if (sig != 0 && pe) return -1;
            *out = pos ? 0.0 : -0.0;
            return 0;
        }
        exp = pe ? exp + e : exp - e;
        if (exp > INT32_MAX) exp = INT32_MAX; /* i32 saturating add/sub */
        if (exp < INT32_MIN) exp = INT32_MIN;
    }
    double f = (double)sig;
    for (;;) {
        const long k = exp < 0 ? -exp : exp;
        if (k <= 308) {
            if (exp >= 0) {
                f *= pow10_tab((int)k);
                if (isinf(f)) return -1; /* NumberOutOfRange */
            } else {
                f /= pow10_tab((int)k);
            }
            break;
        }
        if (f == 0.0) break;
        if (exp >= 0) return -1;
        f /= 1e308;
        exp += 308;
    }
    *out = pos ? f : -f;
    return 0;
}

static void put_utf8(char *o, size_t *k, uint32_t cp) {
    if (cp < 0x80) o[(*k)++] = (char)cp;
    else if (cp < 0x800) {
        o[(*k)++] = (char)(0xC0 | (cp >> 6));
        o[(*k)++] = (char)(0x80 | (cp & 63));
    } else if (cp < 0x10000) {
        o[(*k)++] = (char)(0xE0 | (cp >> 12));
        o[(*k)++] = (char)(0x80 | ((cp >> 6) & 63));
        o[(*k)++] = (char)(0x80 | (cp & 63));
    } else {
        o[(*k)++] = (char)(0xF0 | (cp >> 18));
        o[(*k)++] = (char)(0x80 | ((cp >> 12) & 63));
        o[(*k)++] = (char)(0x80 | ((cp >> 6) & 63));
        o[(*k)++] = (char)(0x80 | (cp & 63));
    }
}

static int hex4(ps *p, uint32_t *v) {
    if (p->i + 4 > p->n) return -1;
    uint32_t x = 0;
    for (int k = 0; k < 4; ++k) {
        char c = p->s[p->i++];
        x <<= 4;
        if (c >= '0' && c <= '9') x |= (uint32_t)(c - '0');
        else if (c >= 'a' && c <= 'f') x |= (uint32_t)(c - 'a' + 10);
        else if (c >= 'A' && c <= 'F') x |= (uint32_t)(c - 'A' + 10);
        else return -1;
    }
    *v = x;
    return 0;
}

static char *str(ps *p, size_t *len) {
    if (p->s[p->i] != '"') { p->err = 1; return NULL; }
    p->i++;
    size_t cap = 16, k = 0;
    char *o = (char *)malloc(cap);
    while (p->i < p->n && p->s[p->i] != '"') {
        if (k + 8 >= cap) { cap *= 2; o = (char *)realloc(o, cap); }
        char c = p->s[p->i++];
        if (c != '\\') { o[k++] = c; continue; }
        if (p->i >= p->n) break;
        c = p->s[p->i++];
        switch (c) {
        case 'n': o[k++] = '\n'; break;
        case 't': o[k++] = '\t'; break;
        case 'r': o[k++] = '\r'; break;
        case 'b': o[k++] = '\b'; break;
        case 'f': o[k++] = '\f'; break;
        case 'u': {
            uint32_t cp;
            if (hex4(p, &cp)) { p->err = 1; free(o); return NULL; }
            if (cp >= 0xD800 && cp < 0xDC00 && p->i + 6 <= p->n && p->s[p->i] == '\\' && p->s[p->i + 1] == 'u') {
                uint32_t lo;
                p->i += 2;
                if (hex4(p, &lo)) { p->err = 1; free(o); return NULL; }
                cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            }
            put_utf8(o, &k, cp);
            break;
        }
        default: o[k++] = c;
        }
    }
    p->i++; /* closing quote */
    o[k] = 0;
    *len = k;
    return o;
}

static void value(ps *p, oj *v);

static void value(ps *p, oj *v) {
    memset(v, 0, sizeof(*v));
    ws(p);
    if (p->i >= p->n) { p->err = 1; return; }
    char c = p->s[p->i];
    if (c == '{' || c == '[') {
        const int obj = c == '{';
        v->kind = obj ? OJ_OBJ : OJ_ARR;
        p->i++;
        size_t cap = 0;
        ws(p);
        if (p->i < p->n && p->s[p->i] == (obj ? '}' : ']')) { p->i++; return; }
        for (;;) {
            if (v->n == cap) {
                cap = cap ? 2 * cap : 4;
                v->items = (oj *)realloc(v->items, cap * sizeof(oj));
                if (obj) {
                    v->keys = (char **)realloc(v->keys, cap * sizeof(char *));
                    v->klens = (size_t *)realloc(v->klens, cap * sizeof(size_t));
                }
            }
            if (obj) {
                ws(p);
                v->keys[v->n] = str(p, &v->klens[v->n]);
                if (p->err) return;
                ws(p);
                if (p->i >= p->n || p->s[p->i] != ':') { p->err = 1; return; }
                p->i++;
            }
            value(p, &v->items[v->n]);
            v->n++;
            if (p->err) return;
            ws(p);
            if (p->i < p->n && p->s[p->i] == ',') { p->i++; continue; }
            if (p->i < p->n && p->s[p->i] == (obj ? '}' : ']')) { p->i++; return; }
            p->err = 1;
            return;
        }
    }
    if (c == '"') {
        v->kind = OJ_STR;
        v->str = str(p, &v->slen);
        return;
    }
    if (!strncmp(p->s + p->i, "true", 4)) { v->kind = OJ_BOOL; v->b = 1; p->i += 4; return; }
    if (!strncmp(p->s + p->i, "false", 5)) { v->kind = OJ_BOOL; p->i += 5; return; }
    if (!strncmp(p->s + p->i, "null", 4)) { v->kind = OJ_NULL; p->i += 4; return; }
    v->kind = OJ_NUM;
    if (serde_number(p, &v->num)) p->err = 1;
}

int orc_json_number(const char *text, size_t n, double *out) {
    ps p = {text, n, 0, 0};
    if (serde_number(&p, out) || p.i != n) return -1;
    return 0;
}

oj *oj_parse(const char *text, size_t n) {
    ps p = {text, n, 0, 0};
    oj *v = (oj *)malloc(sizeof(oj));
    value(&p, v);
    if (p.err) { oj_free(v); return NULL; }
    return v;
}

static void clear(oj *v) {
    for (size_t i = 0; i < v->n; ++i) {
        clear(&v->items[i]);
        if (v->keys) free(v->keys[i]);
    }
    free(v->items);
    free(v->keys);
    free(v->klens);
    free(v->str);
}

void oj_free(oj *v) {
    if (!v) return;
    clear(v);
    free(v);
}

const oj *oj_get(const oj *o, const char *key) {
    if (!o || o->kind != OJ_OBJ) return NULL;
    size_t l = strlen(key);
    for (size_t i = 0; i < o->n; ++i)
        if (o->klens[i] == l && !memcmp(o->keys[i], key, l)) return &o->items[i];
    return NULL;
}
