/* orc_json.c -- minimal JSON parser for the CPU oracle (TEST INFRASTRUCTURE ONLY). */
#include "orc_json.h"

#include <stdint.h>
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
    char *end;
    v->kind = OJ_NUM;
    v->num = strtod(p->s + p->i, &end);
    if (end == p->s + p->i) { p->err = 1; return; }
    p->i = (size_t)(end - p->s);
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
