/*
 * orc_pickle.c -- CPU restatement of the Transport's batch serialisation.
 * TEST INFRASTRUCTURE ONLY (see sdl_oracle.h): the checker for
 * sdl_pickle_frames_device and the CPU baseline of bench.py --frames.
 *
 * The reference Transport sends every finished DataSet as
 * serde_pickle::to_vec(&x, Default::default()) (rust/src/transport/zmq_transmit.rs:71),
 * which the Python consumer reads with pickle.loads (python/external_dataset.py:52).
 * The serializer is the crate serde-pickle 1.1.1 (rust/Cargo.lock:2013-2016; not
 * vendored, not buildable here), restated from its published ser.rs:
 *   to_vec         : PROTO 3 ("\x80\x03"), the value, STOP (".")
 *   struct / map   : EMPTY_DICT "}", MARK "(" when it has fields, per field the key
 *                    then the value, SETITEMS "u" after every 1000 entries
 *                    (followed by a new MARK) and at the end
 *   str (keys)     : BINUNICODE "X" + u32 LE length + UTF-8 bytes
 *   Vec / seq      : EMPTY_LIST "]", and when not empty MARK "(", the elements,
 *                    APPENDS "e" + MARK "(" after every 1000, APPENDS "e" at the end
 *   u32 / i32      : BININT "J" + i32 LE (every id, mask and label fits)
 *   f32 (-> f64)   : BINFLOAT "G" + f64 big-endian
 * The field order and names are the reference's Serialize impls:
 *   BertData (models/bert_data.rs:106-145): input_ids, attention_mask, token_type_ids,
 *     labels (Mask: Vec<Vec<i32>>; MultiLabel: Vec<Vec<f32>>) or, for SingleClass,
 *     label (Vec<u32>), having one entry per filled row (BertData.label is pushed per
 *     row, :50/:75/:80);
 *   GptData (models/gpt_data.rs:53-62): input_ids, attention_mask, labels;
 *   T5Data  (models/t5_data.rs:235-249): input_ids, attention_mask, labels (S/4 wide).
 * Byte-exactness against the crate itself is unpinned (it cannot run here); the
 * bytes are pinned to the consumer's semantics by tests/test_pickle_frames.py
 * (CPython pickle.loads of every frame equals the DataSet's dict).
 */
#include <stdint.h>
#include <string.h>

#include "sdl_oracle.h"

typedef struct {
    uint8_t *p;
    size_t n, cap;
} pw;

static void put(pw *w, const void *s, size_t n) {
    if (w->n + n <= w->cap) memcpy(w->p + w->n, s, n);
    w->n += n;
}
static void put1(pw *w, uint8_t c) { put(w, &c, 1); }

static void put_i32(pw *w, int32_t v) {
    uint8_t b[5] = {'J', (uint8_t)v, (uint8_t)(v >> 8), (uint8_t)(v >> 16), (uint8_t)((uint32_t)v >> 24)};
    put(w, b, 5);
}

static void put_f64(pw *w, double d) {
    uint64_t u;
    memcpy(&u, &d, 8);
    uint8_t b[9];
    b[0] = 'G';
    for (int i = 0; i < 8; ++i) b[1 + i] = (uint8_t)(u >> (56 - 8 * i));
    put(w, b, 9);
}

static void put_key(pw *w, const char *k) {
    uint32_t n = (uint32_t)strlen(k);
    uint8_t b[5] = {'X', (uint8_t)n, (uint8_t)(n >> 8), (uint8_t)(n >> 16), (uint8_t)(n >> 24)};
    put(w, b, 5);
    put(w, k, n);
}

/* serialize_seq + SerializeSeq::{serialize_element, end} */
static void seq_open(pw *w, size_t len) {
    put1(w, ']');
    if (len) put1(w, '(');
}
static void seq_elem_done(pw *w, size_t *count) {
    if (++*count == 1000) {
        put(w, "e(", 2);
        *count = 0;
    }
}
static void seq_close(pw *w, size_t len) {
    if (len) put1(w, 'e');
}

/* Vec<Vec<u32|i32>> of `rows` rows of width `w_` */
static void put_rows_i32(pw *w, const int32_t *a, size_t rows, size_t width) {
    size_t oc = 0;
    seq_open(w, rows);
    for (size_t r = 0; r < rows; ++r) {
        size_t ic = 0;
        seq_open(w, width);
        for (size_t k = 0; k < width; ++k) {
            put_i32(w, a[r * width + k]);
            seq_elem_done(w, &ic);
        }
        seq_close(w, width);
        seq_elem_done(w, &oc);
    }
    seq_close(w, rows);
}

static void put_rows_f32(pw *w, const float *a, size_t rows, size_t width) {
    size_t oc = 0;
    seq_open(w, rows);
    for (size_t r = 0; r < rows; ++r) {
        size_t ic = 0;
        seq_open(w, width);
        for (size_t k = 0; k < width; ++k) {
            put_f64(w, (double)a[r * width + k]);
            seq_elem_done(w, &ic);
        }
        seq_close(w, width);
        seq_elem_done(w, &oc);
    }
    seq_close(w, rows);
}

size_t orc_pickle_dataset(int task, int batch_size, int seq_len, int label_width, int rows, const int32_t *input_ids,
                          const int32_t *attention_mask, const int32_t *token_type_ids, const int32_t *labels,
                          const float *labels_f32, uint8_t *out, size_t cap) {
    pw w = {out, 0, out ? cap : 0};
    const size_t B = (size_t)batch_size, S = (size_t)seq_len, LW = (size_t)label_width;
    const int bert = task == 0 || task == 3 || task == 4; /* MLM / MULTI_LABEL / SINGLE_CLASS -> BertData */
    put(&w, "\x80\x03", 2);
    put1(&w, '}');
    put1(&w, '('); /* every DataSet struct has fields */
    put_key(&w, "input_ids");
    put_rows_i32(&w, input_ids, B, S);
    put_key(&w, "attention_mask");
    put_rows_i32(&w, attention_mask, B, S);
    if (bert) {
        put_key(&w, "token_type_ids");
        put_rows_i32(&w, token_type_ids, B, S);
    }
    if (task == 4) { /* SingleClass: "label": Vec<u32>, one per filled row (bert_data.rs:118-121) */
        size_t c = 0;
        put_key(&w, "label");
        seq_open(&w, (size_t)rows);
        for (int r = 0; r < rows; ++r) {
            put_i32(&w, labels[r]);
            seq_elem_done(&w, &c);
        }
        seq_close(&w, (size_t)rows);
        put1(&w, 'u');
        put1(&w, '.');
        return w.n;
    }
    put_key(&w, "labels");
    if (task == 3)
        put_rows_f32(&w, labels_f32, (size_t)rows, LW);
    else
        put_rows_i32(&w, labels, bert ? (size_t)rows : B, LW);
    put1(&w, 'u');
    put1(&w, '.');
    return w.n;
}
