/* orc_json.h -- minimal JSON tree for reading HF tokenizer.json in the CPU
 * oracle (TEST INFRASTRUCTURE ONLY). Objects keep file order. */
#ifndef ORC_JSON_H
#define ORC_JSON_H
#include <stddef.h>

typedef enum { OJ_NULL, OJ_BOOL, OJ_NUM, OJ_STR, OJ_ARR, OJ_OBJ } oj_kind;

typedef struct oj {
    oj_kind kind;
    int b;
    double num;
    char *str;        /* OJ_STR: UTF-8, NUL-terminated; len in slen */
    size_t slen;
    struct oj *items; /* OJ_ARR / OJ_OBJ values */
    char **keys;      /* OJ_OBJ keys */
    size_t *klens;
    size_t n;
} oj;

/* Parses text[0..n); NULL on error. */
oj *oj_parse(const char *text, size_t n);
void oj_free(oj *v);
/* One JSON number as serde_json 1.0.87 parses it into an f64 (default
 * features); 0 ok, -1 not a number / out of range. */
int orc_json_number(const char *text, size_t n, double *out);
const oj *oj_get(const oj *obj, const char *key);
#endif
