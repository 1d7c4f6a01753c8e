/* orc_internal.h -- shared pieces of the CPU oracle (TEST INFRASTRUCTURE ONLY). */
#ifndef ORC_INTERNAL_H
#define ORC_INTERNAL_H
#include <stdlib.h>
#include "sdl_oracle.h"

typedef struct {
    uint32_t *p;
    size_t n, cap;
} idvec;

static inline void idpush(idvec *v, uint32_t x) {
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 256;
        v->p = (uint32_t *)realloc(v->p, v->cap * sizeof(uint32_t));
    }
    v->p[v->n++] = x;
}

/* Tokenizer::encode(text, true).get_ids() of one tokenizer kind, plus the
 * TokenizerWrapper::encode_mask framing ids around it (tokenizer_wrapper.rs:107-134). */
struct orc_encoder {
    void (*encode)(const void *impl, const uint8_t *s, size_t n, idvec *out);
    const void *impl;
    int npre, npost;
    uint32_t pre[4], post[4];
    uint32_t extra[100]; /* T5 <extra_id_k> ids (TokenizerInfo.extra, tokenizer_wrapper.rs:77-80) */
};

void orc_bert_encode_vec(const orc_tok *t, const uint8_t *s, size_t n, idvec *out);
#endif
