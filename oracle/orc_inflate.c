/* orc_inflate.c -- CPU oracle (TEST INFRASTRUCTURE ONLY: loaded by tests/ as the
 * checker, never by the product) for the provider's gzip inflate.
 *
 * The reference reads `.json.gz` files through async-compression 0.3.14's
 * GzipDecoder over flate2 1.0.24 / miniz_oxide 0.5.4 (rust/Cargo.lock;
 * gzip_file_provider.rs:13-28) -- third-party crates, not vendored, not
 * buildable here (no cargo).  DEFLATE decoding is fully specified by RFC 1951
 * (and the member framing by RFC 1952), so this is a direct restatement of the
 * RFCs in the style of Mark Adler's puff (bit-serial canonical Huffman decode),
 * with zlib's error rules (incomplete/over-subscribed codes, missing end-of-block
 * code, bad repeats, invalid codes, distance too far back, stored LEN/NLEN, header
 * flags/CRC, trailer CRC-32 and ISIZE).  Pinned by tests/test_inflate.py against
 * CPython's zlib on streams of every block type and on the reference's own
 * data/test.json.gz (tests/golden/test.json.gz).  Status codes match the
 * device's GZ_* codes (csrc/kernels.hpp).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

enum { OK = 0, E_RANGE, E_TRUNC, E_HEADER, E_HCRC, E_BTYPE, E_STORED, E_CODES, E_CODE, E_FAR, E_OVER, E_SIZE, E_TRAIL, E_CRC };

typedef struct {
    const uint8_t *in;
    size_t inlen, pos;   /* byte position */
    uint32_t bitbuf;
    int bitcnt;
    uint8_t *out;
    size_t outcap, outpos;
    int err;
} St;

static int bits(St *s, int need) {
    uint32_t v = s->bitbuf;
    while (s->bitcnt < need) {
        if (s->pos >= s->inlen) {
            s->err = E_TRUNC;
            return 0;
        }
        v |= (uint32_t)s->in[s->pos++] << s->bitcnt;
        s->bitcnt += 8;
    }
    s->bitbuf = v >> need;
    s->bitcnt -= need;
    return (int)(v & ((1u << need) - 1u));
}

typedef struct {
    short count[16];
    short symbol[320];
} Huff;

/* canonical decode, one bit at a time (RFC 1951 3.2.2) */
static int decode(St *s, const Huff *h) {
    int code = 0, first = 0, index = 0;
    for (int len = 1; len <= 15; ++len) {
        code |= bits(s, 1);
        if (s->err) return -1;
        int count = h->count[len];
        if (code - count < first) return h->symbol[index + (code - first)];
        index += count;
        first += count;
        first <<= 1;
        code <<= 1;
    }
    return -2; /* ran out of codes */
}

/* returns the number of unused codes (0 complete, > 0 incomplete, < 0 over-subscribed) */
static int construct(Huff *h, const short *length, int n, int *maxlen) {
    short offs[16];
    memset(h->count, 0, sizeof(h->count));
    for (int s = 0; s < n; ++s) h->count[length[s]]++;
    *maxlen = 0;
    for (int l = 1; l < 16; ++l)
        if (h->count[l]) *maxlen = l;
    if (h->count[0] == n) return 0; /* no codes */
    int left = 1;
    for (int l = 1; l < 16; ++l) {
        left <<= 1;
        left -= h->count[l];
        if (left < 0) return left;
    }
    offs[1] = 0;
    for (int l = 1; l < 15; ++l) offs[l + 1] = offs[l] + h->count[l];
    for (int s = 0; s < n; ++s)
        if (length[s]) h->symbol[offs[length[s]]++] = (short)s;
    return left;
}

static const short LBASE[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const short LEXT[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const short DBASE[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const short DEXT[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

static int codes(St *s, const Huff *lc, const Huff *dc) {
    for (;;) {
        int sym = decode(s, lc);
        if (s->err) return s->err;
        if (sym < 0) return E_CODE;
        if (sym < 256) {
            if (s->outpos >= s->outcap) return E_OVER;
            s->out[s->outpos++] = (uint8_t)sym;
        } else if (sym == 256) {
            return OK;
        } else {
            sym -= 257;
            if (sym >= 29) return E_CODE;
            int len = LBASE[sym] + bits(s, LEXT[sym]);
            if (s->err) return s->err;
            int ds = decode(s, dc);
            if (s->err) return s->err;
            if (ds < 0 || ds >= 30) return E_CODE;
            size_t dist = (size_t)(DBASE[ds] + bits(s, DEXT[ds]));
            if (s->err) return s->err;
            if (dist > s->outpos) return E_FAR;
            if (s->outpos + (size_t)len > s->outcap) return E_OVER;
            while (len--) {
                s->out[s->outpos] = s->out[s->outpos - dist];
                s->outpos++;
            }
        }
    }
}

static int fixed_block(St *s) {
    static Huff lc, dc;
    static int built = 0;
    if (!built) {
        short l[320];
        int mx;
        for (int i = 0; i < 288; ++i) l[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
        construct(&lc, l, 288, &mx);
        for (int i = 0; i < 30; ++i) l[i] = 5;
        construct(&dc, l, 30, &mx);
        built = 1;
    }
    return codes(s, &lc, &dc);
}

static int dynamic_block(St *s) {
    static const short order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    short lengths[320];
    Huff lc, dc;
    int mx;
    int nlen = bits(s, 5) + 257, ndist = bits(s, 5) + 1, ncode = bits(s, 4) + 4;
    if (s->err) return s->err;
    if (nlen > 286 || ndist > 30) return E_CODES;
    int idx;
    for (idx = 0; idx < ncode; ++idx) lengths[order[idx]] = (short)bits(s, 3);
    for (; idx < 19; ++idx) lengths[order[idx]] = 0;
    if (s->err) return s->err;
    if (construct(&lc, lengths, 19, &mx) != 0 || mx == 0) return E_CODES; /* must be complete */
    idx = 0;
    while (idx < nlen + ndist) {
        int sym = decode(s, &lc);
        if (s->err) return s->err;
        if (sym < 0) return E_CODES;
        if (sym < 16) {
            lengths[idx++] = (short)sym;
        } else {
            short len = 0;
            int rep;
            if (sym == 16) {
                if (idx == 0) return E_CODES;
                len = lengths[idx - 1];
                rep = 3 + bits(s, 2);
            } else if (sym == 17) {
                rep = 3 + bits(s, 3);
            } else {
                rep = 11 + bits(s, 7);
            }
            if (s->err) return s->err;
            if (idx + rep > nlen + ndist) return E_CODES;
            while (rep--) lengths[idx++] = len;
        }
    }
    if (lengths[256] == 0) return E_CODES;
    int left = construct(&lc, lengths, nlen, &mx);
    if (left < 0 || (left > 0 && mx != 1)) return E_CODES;
    left = construct(&dc, lengths + nlen, ndist, &mx);
    if (left < 0 || (left > 0 && mx > 1)) return E_CODES;
    return codes(s, &lc, &dc);
}

static uint32_t crc32_update(uint32_t c, const uint8_t *p, size_t n) {
    c = ~c;
    while (n--) {
        c ^= *p++;
        for (int k = 0; k < 8; ++k) c = c & 1u ? (c >> 1) ^ 0xEDB88320u : c >> 1;
    }
    return ~c;
}

/* ISIZE of one member from its last 4 bytes (0 for a bad or short member) */
uint32_t orc_gz_isize(const uint8_t *m, size_t n) {
    if (n < 18) return 0;
    return (uint32_t)m[n - 4] | (uint32_t)m[n - 3] << 8 | (uint32_t)m[n - 2] << 16 | (uint32_t)m[n - 1] << 24;
}

/* Inflates one gzip member m[0..n) into out (capacity cap = its ISIZE);
 * *produced = bytes written.  Returns a status code (0 ok). */
int orc_gz_inflate(const uint8_t *m, size_t n, uint8_t *out, size_t cap, size_t *produced) {
    *produced = 0;
    if (n < 18) return E_TRUNC;
    if (m[0] != 0x1f || m[1] != 0x8b || m[2] != 8) return E_HEADER;
    /* The product sizes each member's output from its trailer before decoding
     * (sdl_gzip_inflate_device), so an ISIZE that DEFLATE cannot reach (more
     * than 1032:1, + 64) fails the member here, ahead of any decode error zlib
     * would report first; which reason a corrupt member gets is the device
     * contract's (GZ_*), the fact that it fails is zlib's. */
    if ((uint64_t)orc_gz_isize(m, n) > 1032ull * n + 64) return E_SIZE;
    const uint8_t flg = m[3];
    if (flg & 0xE0) return E_HEADER;
    size_t p = 10;
    if (flg & 4) {
        if (p + 2 > n) return E_TRUNC;
        p += 2 + ((size_t)m[p] | (size_t)m[p + 1] << 8);
    }
    for (int f = 8; f <= 16; f <<= 1)
        if (flg & f) {
            while (p < n && m[p]) ++p;
            ++p;
        }
    if (flg & 2) {
        if (p + 2 > n) return E_TRUNC;
        if ((crc32_update(0, m, p) & 0xFFFFu) != ((uint32_t)m[p] | (uint32_t)m[p + 1] << 8)) return E_HCRC;
        p += 2;
    }
    if (p + 8 > n) return E_TRUNC;
    St s = {m, n - 8, p, 0, 0, out, cap, 0, OK};
    int last;
    do {
        last = bits(&s, 1);
        int type = bits(&s, 2);
        if (s.err) return s.err;
        int rc;
        if (type == 0) {
            s.bitbuf = 0;
            s.bitcnt = 0;
            if (s.pos + 4 > s.inlen) return E_TRUNC;
            unsigned len = s.in[s.pos] | s.in[s.pos + 1] << 8, nlen = s.in[s.pos + 2] | s.in[s.pos + 3] << 8;
            s.pos += 4;
            if (len != (~nlen & 0xFFFFu)) return E_STORED;
            if (s.pos + len > s.inlen) return E_TRUNC;
            if (s.outpos + len > s.outcap) return E_OVER;
            memcpy(s.out + s.outpos, s.in + s.pos, len);
            s.outpos += len;
            s.pos += len;
            rc = OK;
        } else if (type == 1) {
            rc = fixed_block(&s);
        } else if (type == 2) {
            rc = dynamic_block(&s);
        } else {
            rc = E_BTYPE;
        }
        *produced = s.outpos;
        if (rc) return rc;
    } while (!last);
    const size_t t = s.pos; /* trailer: the bit buffer holds no whole unread byte */
    if (t + 8 != n) return E_TRAIL;
    const uint32_t crc = (uint32_t)m[t] | (uint32_t)m[t + 1] << 8 | (uint32_t)m[t + 2] << 16 | (uint32_t)m[t + 3] << 24;
    const uint32_t isz = (uint32_t)m[t + 4] | (uint32_t)m[t + 5] << 8 | (uint32_t)m[t + 6] << 16 | (uint32_t)m[t + 7] << 24;
    if (isz != (uint32_t)s.outpos || s.outpos != cap) return E_SIZE;
    if (crc32_update(0, out, s.outpos) != crc) return E_CRC;
    return OK;
}
