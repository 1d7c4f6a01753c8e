// json_text.hip -- the Data Provider's JsonText filter on gfx950 (SURVEY.md
// §8(f) row 2: the step that feeds the Batcher's text arena).
//
// Restates, for a whole buffer of inflated JSON lines at once, what the
// reference's gzip/zstd providers do one line at a time
// (gzip_file_provider.rs:30-50 / zstd_file_provider.rs:23-45 ->
// SourceFilter::JsonText, source_filter.rs:15-20 -> provider_util.rs:60-64
// create_json_text: serde_json::from_str(&line).unwrap(), v["text"].as_str()):
//   - lines are split on '\n' (tokio lines(); a trailing '\r' is JSON
//     whitespace here, as are ' ' and '\t');
//   - a line whose value is an object with a string member "text" (the last one
//     when the key repeats: serde_json's map keeps the last) yields one record,
//     that string unescaped to UTF-8; a valid line without one yields nothing;
//   - a line the reference's unwrap() would panic on (invalid JSON or UTF-8,
//     nesting past serde_json's recursion limit of 128, lone surrogate escapes)
//     yields nothing and is counted.
// Numbers are checked for JSON syntax only: a literal beyond the f64 range,
// which serde_json rejects, is accepted (known divergences).
//
// Layout: one lane per line.  A line is read forward through 16-B loads of its
// aligned blocks (the buffer is 16-B aligned and readable to a multiple of 16
// bytes), parsed by an iterative state machine with a 128-bit container stack
// in registers, and only the chosen string's raw span and decoded length are
// kept.  After two scans (decoded lengths -> text offsets, record flags ->
// record indices) a second lane-per-line pass decodes the spans into the arena.
// Lines are independent and short relative to the buffer, so thousands of
// lanes run at once; newline positions come from a wave-per-KiB count + scan.
#include "common.hpp"
#include "device_util.hpp"
#include "kernels.hpp"

namespace sdl {

namespace {

constexpr int JSON_MAX_DEPTH = 127;  // serde_json: remaining_depth 128, an error when it reaches 0
constexpr int JL_MIN_LANE = 512;     // lines this long go to the wave kernels (= JL_MIN)

// forward reader over one lane's line: 16-B loads of aligned blocks
struct LaneReader {
    const uint8_t *base;
    int64_t blk;
    uint4 v;
    __device__ uint32_t at(int64_t p) {
        const int64_t b = p & ~(int64_t)15;
        if (b != blk) {
            blk = b;
            v = *reinterpret_cast<const uint4 *>(base + b);
        }
        const int k = (int)(p & 15);
        const uint32_t w = k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w;
        return (w >> (8 * (k & 3))) & 0xFFu;
    }
};

__device__ __forceinline__ bool json_ws(uint32_t c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }
__device__ __forceinline__ int hexval(uint32_t c) {
    if (c - '0' < 10u) return (int)(c - '0');
    if ((c | 0x20u) - 'a' < 6u) return (int)((c | 0x20u) - 'a' + 10);
    return -1;
}
__device__ __forceinline__ int utf8_len_cp(uint32_t cp) { return cp < 0x80u ? 1 : cp < 0x800u ? 2 : cp < 0x10000u ? 3 : 4; }

// Parses the JSON string whose opening quote is at p - 1; p is left after the
// closing quote.  Returns false on any error serde_json reports (control char,
// bad escape, lone surrogate, invalid UTF-8, end of line).  *out_len = decoded
// UTF-8 bytes; when key != null, *is_text = the decoded string equals "text".
__device__ bool json_string(LaneReader &rd, int64_t &p, int64_t le, uint32_t *out_len, bool want_key, bool *is_text) {
    uint32_t n = 0;
    bool match = want_key;
    auto emit = [&](uint32_t byte) {
        if (want_key) match = match && n < 4 && byte == (uint32_t)"text"[n];
        ++n;
    };
    for (;;) {
        if (p >= le) return false;
        const uint32_t c = rd.at(p++);
        if (c == '"') break;
        if (c < 0x20u) return false;
        if (c == '\\') {
            if (p >= le) return false;
            const uint32_t e = rd.at(p++);
            uint32_t cp;
            if (e == '"' || e == '\\' || e == '/') cp = e;
            else if (e == 'b') cp = 8;
            else if (e == 'f') cp = 12;
            else if (e == 'n') cp = 10;
            else if (e == 'r') cp = 13;
            else if (e == 't') cp = 9;
            else if (e == 'u') {
                auto hex4 = [&](uint32_t *v) -> bool {
                    if (p + 4 > le) return false;
                    uint32_t x = 0;
                    for (int k = 0; k < 4; ++k) {
                        const int h = hexval(rd.at(p++));
                        if (h < 0) return false;
                        x = x << 4 | (uint32_t)h;
                    }
                    *v = x;
                    return true;
                };
                if (!hex4(&cp)) return false;
                if (cp >= 0xDC00u && cp <= 0xDFFFu) return false;  // lone trailing surrogate
                if (cp >= 0xD800u && cp <= 0xDBFFu) {                // must pair with \uDC00-DFFF
                    if (p + 2 > le || rd.at(p) != '\\' || rd.at(p + 1) != 'u') return false;
                    p += 2;
                    uint32_t lo;
                    if (!hex4(&lo) || lo < 0xDC00u || lo > 0xDFFFu) return false;
                    cp = 0x10000u + ((cp - 0xD800u) << 10) + (lo - 0xDC00u);
                }
            } else {
                return false;
            }
            // the decoded code point's UTF-8 bytes
            const int l = utf8_len_cp(cp);
            if (!want_key) {
                n += (uint32_t)l;
            } else if (l == 1) {
                emit(cp);
            } else {
                for (int k = 0; k < l; ++k) emit(0x80u);  // never matches "text"
            }
            continue;
        }
        if (c < 0x80u) {
            emit(c);
            continue;
        }
        // UTF-8 sequence (a Rust String: strict)
        int l;
        uint32_t cp, mn;
        if ((c & 0xE0u) == 0xC0u) { l = 2; cp = c & 0x1Fu; mn = 0x80u; }
        else if ((c & 0xF0u) == 0xE0u) { l = 3; cp = c & 0x0Fu; mn = 0x800u; }
        else if ((c & 0xF8u) == 0xF0u) { l = 4; cp = c & 0x07u; mn = 0x10000u; }
        else return false;
        if (p + l - 1 > le) return false;
        for (int k = 1; k < l; ++k) {
            const uint32_t x = rd.at(p++);
            if ((x & 0xC0u) != 0x80u) return false;
            cp = cp << 6 | (x & 0x3Fu);
        }
        if (cp < mn || cp > 0x10FFFFu || (cp >= 0xD800u && cp <= 0xDFFFu)) return false;
        for (int k = 0; k < l; ++k) emit(0x80u);
    }
    *out_len = n;
    if (want_key) *is_text = match && n == 4;
    return true;
}

// JSON number at p (first char '-' or a digit); p is left after it
__device__ bool json_number(LaneReader &rd, int64_t &p, int64_t le) {
    auto digit = [&](int64_t q) { return q < le && rd.at(q) - '0' < 10u; };
    if (rd.at(p) == '-') ++p;
    if (!digit(p)) return false;
    if (rd.at(p) == '0') {
        ++p;
    } else {
        while (digit(p)) ++p;
    }
    if (p < le && rd.at(p) == '.') {
        ++p;
        if (!digit(p)) return false;
        while (digit(p)) ++p;
    }
    if (p < le && (rd.at(p) | 0x20u) == 'e') {
        ++p;
        if (p < le && (rd.at(p) == '+' || rd.at(p) == '-')) ++p;
        if (!digit(p)) return false;
        while (digit(p)) ++p;
    }
    return true;
}

enum : int { M_VALUE = 0, M_AFTER = 1, M_KEY = 2 };

}  // namespace

// ---------------------------------------------------------------------------
// Newline positions: one wave per KiB, lane t owns 16 bytes.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_json_nl_count(const uint8_t *__restrict__ buf, int64_t len,
                                                      uint32_t *__restrict__ cnt) {
    const int64_t p0 = (int64_t)blockIdx.x * CHUNK + 16 * threadIdx.x;
    uint32_t c = 0;
    if (p0 < len) {
        const uint4 v = *reinterpret_cast<const uint4 *>(buf + p0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        for (int i = 0; i < 16 && p0 + i < len; ++i) c += ((w[i >> 2] >> (8 * (i & 3))) & 0xFFu) == '\n';
    }
    const uint32_t incl = wave_incl_sum(c);
    if (threadIdx.x == 63) cnt[blockIdx.x] = incl;
}

__global__ __launch_bounds__(64) void k_json_nl_write(const uint8_t *__restrict__ buf, int64_t len,
                                                      const uint32_t *__restrict__ base, uint32_t *__restrict__ nl,
                                                      uint32_t cap) {
    const int64_t p0 = (int64_t)blockIdx.x * CHUNK + 16 * threadIdx.x;
    uint32_t m = 0;
    if (p0 < len) {
        const uint4 v = *reinterpret_cast<const uint4 *>(buf + p0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        for (int i = 0; i < 16 && p0 + i < len; ++i) m |= (((w[i >> 2] >> (8 * (i & 3))) & 0xFFu) == '\n' ? 1u : 0u) << i;
    }
    const uint32_t c = (uint32_t)__builtin_popcount(m);
    uint32_t at = base[blockIdx.x] + wave_incl_sum(c) - c;
    for (; m; m &= m - 1, ++at)  // past `cap` the host grows the list and writes it again
        if (at < cap) nl[at] = (uint32_t)(p0 + __builtin_ctz(m));
}

// line i = [start, end): after newline i - 1 up to newline i (or the end)
__device__ __forceinline__ void line_span(const uint32_t *nl, uint32_t n_nl, int64_t len, int64_t i, int64_t *s,
                                          int64_t *e) {
    *s = i == 0 ? 0 : (int64_t)nl[i - 1] + 1;
    *e = i < (int64_t)n_nl ? (int64_t)nl[i] : len;
}

// ---------------------------------------------------------------------------
// Parse: one lane per line -> (raw span of the chosen string, decoded length).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_json_parse(const uint8_t *__restrict__ buf, int64_t len,
                                                    const uint32_t *__restrict__ nl, uint32_t n_nl, int64_t n_lines,
                                                    uint32_t *__restrict__ out_len, uint32_t *__restrict__ is_rec,
                                                    uint2 *__restrict__ span, uint32_t *__restrict__ n_invalid) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_lines) return;
    int64_t p, le;
    line_span(nl, n_nl, len, i, &p, &le);
    if (le - p >= JL_MIN_LANE) return;  // a wave parses it (k_json_parse_long)
    LaneReader rd{buf, -1, make_uint4(0, 0, 0, 0)};
    uint64_t stk0 = 0, stk1 = 0;  // bit d: the container at depth d + 1 is an object
    int depth = 0;
    int mode = M_VALUE;
    bool key_text = false;        // the member being parsed is the top-level "text"
    bool found = false, ok = true;
    uint32_t f_len = 0, f_s = 0, f_e = 0;
    auto is_obj = [&](int d) -> bool {  // container at depth d (>= 1)
        const int b = d - 1;
        return b < 64 ? (stk0 >> b) & 1ull : (stk1 >> (b - 64)) & 1ull;
    };
    for (;;) {
        while (p < le && json_ws(rd.at(p))) ++p;
        if (mode == M_AFTER && depth == 0) {
            ok = p == le;  // trailing characters
            break;
        }
        if (p >= le) { ok = false; break; }
        const uint32_t c = rd.at(p);
        if (mode == M_VALUE) {
            const bool member_text = key_text;
            key_text = false;
            if (c == '{' || c == '[') {
                if (depth >= JSON_MAX_DEPTH) { ok = false; break; }
                const uint64_t bit = c == '{' ? 1ull : 0ull;
                if (depth < 64) stk0 = (stk0 & ~(1ull << depth)) | (bit << depth);
                else stk1 = (stk1 & ~(1ull << (depth - 64))) | (bit << (depth - 64));
                ++depth;
                ++p;
                if (member_text) found = false;  // "text" is not a string: as_str() is None
                while (p < le && json_ws(rd.at(p))) ++p;
                if (p < le && rd.at(p) == (c == '{' ? '}' : ']')) {
                    ++p;
                    --depth;
                    mode = M_AFTER;
                } else {
                    mode = c == '{' ? M_KEY : M_VALUE;
                }
                continue;
            }
            if (c == '"') {
                const int64_t s = ++p;
                uint32_t n;
                if (!json_string(rd, p, le, &n, false, nullptr)) { ok = false; break; }
                if (member_text) {
                    found = true;
                    f_len = n;
                    f_s = (uint32_t)s;
                    f_e = (uint32_t)(p - 1);
                }
                mode = M_AFTER;
                continue;
            }
            if (member_text) found = false;
            if (c == '-' || c - '0' < 10u) {
                if (!json_number(rd, p, le)) { ok = false; break; }
                mode = M_AFTER;
                continue;
            }
            const char *lit = c == 't' ? "true" : c == 'f' ? "false" : c == 'n' ? "null" : nullptr;
            if (!lit) { ok = false; break; }
            int k = 0;
            for (; lit[k]; ++k)
                if (p + k >= le || rd.at(p + k) != (uint32_t)lit[k]) break;
            if (lit[k]) { ok = false; break; }
            p += k;
            mode = M_AFTER;
            continue;
        }
        if (mode == M_KEY) {  // a member name, then ':'
            if (c != '"') { ok = false; break; }
            ++p;
            uint32_t n;
            bool is_text = false;
            if (!json_string(rd, p, le, &n, depth == 1, &is_text)) { ok = false; break; }
            while (p < le && json_ws(rd.at(p))) ++p;
            if (p >= le || rd.at(p) != ':') { ok = false; break; }
            ++p;
            key_text = depth == 1 && is_text;
            mode = M_VALUE;
            continue;
        }
        // M_AFTER inside a container: ',' or its closer
        const bool obj = is_obj(depth);
        if (c == ',') {
            ++p;
            mode = obj ? M_KEY : M_VALUE;
            continue;
        }
        if (c == (obj ? '}' : ']')) {
            ++p;
            --depth;
            mode = M_AFTER;
            continue;
        }
        ok = false;
        break;
    }
    // the top-level value must be an object for v["text"] to be a member
    const bool rec = ok && found;
    out_len[i] = rec ? f_len : 0u;
    is_rec[i] = rec ? 1u : 0u;
    span[i] = make_uint2(f_s, f_e);
    if (!ok) atomicAdd(n_invalid, 1u);
}

// ---------------------------------------------------------------------------
// Decode: one lane per record line -> its UTF-8 bytes at its text offset.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_json_write(const uint8_t *__restrict__ buf, const uint32_t *__restrict__ nl,
                                                    uint32_t n_nl, int64_t len, int64_t n_lines,
                                                    const uint32_t *__restrict__ is_rec, const uint2 *__restrict__ span,
                                                    const uint32_t *__restrict__ toff, const uint32_t *__restrict__ ridx,
                                                    uint8_t *__restrict__ text, uint64_t *__restrict__ offsets) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_lines) return;
    if (i == n_lines - 1) offsets[ridx[n_lines]] = toff[n_lines];  // offsets[n_records] = total bytes
    if (!is_rec[i]) return;
    offsets[ridx[i]] = toff[i];
    {
        int64_t ls, le;
        line_span(nl, n_nl, len, i, &ls, &le);
        if (le - ls >= JL_MIN_LANE) return;  // a wave decodes it (k_json_write_long)
    }
    LaneReader rd{buf, -1, make_uint4(0, 0, 0, 0)};
    uint8_t *o = text + toff[i];
    const int64_t e = span[i].y;
    for (int64_t p = span[i].x; p < e;) {
        const uint32_t c = rd.at(p++);
        if (c != '\\') {
            *o++ = (uint8_t)c;
            continue;
        }
        const uint32_t x = rd.at(p++);
        uint32_t cp = x == 'b' ? 8u : x == 'f' ? 12u : x == 'n' ? 10u : x == 'r' ? 13u : x == 't' ? 9u : x;
        if (x == 'u') {
            auto hex4 = [&]() {
                uint32_t v = 0;
                for (int k = 0; k < 4; ++k) v = v << 4 | (uint32_t)hexval(rd.at(p++));
                return v;
            };
            cp = hex4();
            if (cp >= 0xD800u && cp <= 0xDBFFu) {  // validated pair
                p += 2;
                cp = 0x10000u + ((cp - 0xD800u) << 10) + (hex4() - 0xDC00u);
            }
        }
        if (cp < 0x80u) {
            *o++ = (uint8_t)cp;
        } else if (cp < 0x800u) {
            *o++ = (uint8_t)(0xC0u | cp >> 6);
            *o++ = (uint8_t)(0x80u | (cp & 0x3Fu));
        } else if (cp < 0x10000u) {
            *o++ = (uint8_t)(0xE0u | cp >> 12);
            *o++ = (uint8_t)(0x80u | ((cp >> 6) & 0x3Fu));
            *o++ = (uint8_t)(0x80u | (cp & 0x3Fu));
        } else {
            *o++ = (uint8_t)(0xF0u | cp >> 18);
            *o++ = (uint8_t)(0x80u | ((cp >> 12) & 0x3Fu));
            *o++ = (uint8_t)(0x80u | ((cp >> 6) & 0x3Fu));
            *o++ = (uint8_t)(0x80u | (cp & 0x3Fu));
        }
    }
}

// ---------------------------------------------------------------------------
// Long lines (>= JL_MIN bytes): one wave per line, 1 KiB per step, lane t owns
// 16 bytes.  Data-parallel per step: the escape state of every byte (parity of
// the backslash run before it, carried across lanes and steps), unescaped
// quotes -> in-string mask (prefix parity), string-content checks (control
// chars, escapes, strict UTF-8) and each byte's decoded length; the bytes
// outside strings and the quotes become tokens (LDS list with the decoded-length
// prefix at each), which lane 0 runs through the same JSON grammar as the lane
// kernel.  A long line is mostly one string, so the sequential part is short.
// ---------------------------------------------------------------------------
constexpr int JL_MIN = 512;
constexpr int JW_PRE = 16;  // previous step's last 16 bytes (UTF-8 look-back)
constexpr int JW_WIN = JW_PRE + CHUNK + 16;  // + next 16 bytes (escape look-ahead)

// A lane's 16 bytes as 16-bit masks.
struct JMask {
    uint32_t v, q, b, c, w, hi;  // in line, '"', '\\', < 0x20, json ws (not \n), >= 0x80
};
__device__ __forceinline__ JMask jmask(const uint4 &x, int64_t p0, int64_t s, int64_t e) {
    JMask m{0, 0, 0, 0, 0, 0};
    const uint32_t wv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t c = (wv[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        const int64_t p = p0 + k;
        const uint32_t in = (p >= s && p < e) ? 1u : 0u;
        m.v |= in << k;
        m.q |= (in & (c == '"' ? 1u : 0u)) << k;
        m.b |= (in & (c == '\\' ? 1u : 0u)) << k;
        m.c |= (in & (c < 0x20u ? 1u : 0u)) << k;
        m.w |= (in & (c == ' ' || c == '\t' || c == '\r' ? 1u : 0u)) << k;
        m.hi |= (in & (c >= 0x80u ? 1u : 0u)) << k;
    }
    return m;
}

// Exclusive "last set wins" scan over the wave: x = 0x100 | bit sets the carry,
// 0 passes through; returns the carry before this lane (0 if none).
__device__ __forceinline__ uint32_t wave_excl_last(uint32_t x) {
    DPP_SCAN(x, last_set);  // (DPP steps, device_util.hpp)
    return wave_prev(x);
}
__device__ __forceinline__ uint32_t xor_op(uint32_t a, uint32_t b) { return a ^ b; }
__device__ __forceinline__ uint32_t wave_excl_xor(uint32_t x) {
    uint32_t v = x;
    DPP_SCAN(v, xor_op);
    return v ^ x;
}

// Per lane: escape-parity mask E (bit k: an odd backslash run precedes byte k)
// given the parity carried into the lane; returns the parity carried out.
__device__ __forceinline__ uint32_t esc_mask(uint32_t b, uint32_t v, uint32_t par, uint32_t *E) {
    uint32_t e = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        e |= par << k;
        par = ((b >> k) & 1u) ? par ^ 1u : 0u;
        par &= (v >> k) & 1u;
    }
    *E = e;
    return par;
}
// the escape parity carried into each lane of a step (wave scan) from `carry`
__device__ __forceinline__ uint32_t esc_carry_in(uint32_t b, uint32_t v, uint32_t carry) {
    // lane summary: all 16 bytes backslashes -> the run passes through (16 is even)
    uint32_t tail = 0;  // parity of the trailing backslash run
    for (int k = 15; k >= 0 && ((b >> k) & 1u); --k) tail ^= 1u;
    const uint32_t allbs = (b == 0xFFFFu && v == 0xFFFFu) ? 1u : 0u;
    const uint32_t x = allbs ? 0u : (0x100u | tail);
    const uint32_t ex = wave_excl_last(x);
    return (ex & 0x100u) ? (ex & 1u) : carry;
}

__device__ __forceinline__ uint32_t lds_at(const uint8_t *w, int i) { return w[i]; }

// escape at window index i (the backslash): consumed bytes (2, 6, 12) and
// decoded UTF-8 length; *bad on a serde_json error; `lim` = window index of
// the line end (bytes past it do not exist)
__device__ __forceinline__ int esc_info(const uint8_t *w, int i, int lim, int *dl, uint32_t *cp_out, bool *bad) {
    if (i + 1 >= lim) { *bad = true; return 2; }
    const uint32_t x = w[i + 1];
    *dl = 1;
    *cp_out = x == 'b' ? 8u : x == 'f' ? 12u : x == 'n' ? 10u : x == 'r' ? 13u : x == 't' ? 9u : x;
    if (x == '"' || x == '\\' || x == '/' || x == 'b' || x == 'f' || x == 'n' || x == 'r' || x == 't') return 2;
    if (x != 'u') { *bad = true; return 2; }
    auto hex4 = [&](int at, uint32_t *val) -> bool {
        if (at + 4 > lim) return false;
        uint32_t v = 0;
        for (int k = 0; k < 4; ++k) {
            const int h = hexval(w[at + k]);
            if (h < 0) return false;
            v = v << 4 | (uint32_t)h;
        }
        *val = v;
        return true;
    };
    uint32_t cp;
    if (!hex4(i + 2, &cp)) { *bad = true; return 6; }
    if (cp >= 0xDC00u && cp <= 0xDFFFu) { *bad = true; return 6; }
    if (cp >= 0xD800u && cp <= 0xDBFFu) {
        uint32_t lo;
        if (i + 8 > lim || w[i + 6] != '\\' || w[i + 7] != 'u' || !hex4(i + 8, &lo) || lo < 0xDC00u || lo > 0xDFFFu) {
            *bad = true;
            return 6;
        }
        *dl = 4;
        *cp_out = 0x10000u + ((cp - 0xD800u) << 10) + (lo - 0xDC00u);
        return 12;
    }
    *dl = utf8_len_cp(cp);
    *cp_out = cp;
    return 6;
}

// bytes an escape at window index i consumes (2, 6, or 12 for a \uD8xx\uDCxx
// pair), without validating it (esc_info does)
__device__ __forceinline__ int esc_len(const uint8_t *w, int i, int lim) {
    if (i + 1 >= lim || w[i + 1] != 'u') return 2;
    if (i + 6 > lim) return 6;
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
        const int h = hexval(w[i + 2 + k]);
        if (h < 0) return 6;
        v = v << 4 | (uint32_t)h;
    }
    return (v >= 0xD800u && v <= 0xDBFFu && i + 8 <= lim && w[i + 6] == '\\' && w[i + 7] == 'u') ? 12 : 6;
}

// Bytes of the escape sequence running out of this lane's 16 bytes into the
// next lane, given `skip` bytes consumed at its start by the previous lane's.
__device__ __forceinline__ uint32_t lane_spill(const uint8_t *w, int wi0, uint32_t ct, uint32_t b, int lim, int skip) {
    if (!(ct & b) && skip == 0) return 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        if (skip > 0) {
            --skip;
        } else if ((ct >> k) & (b >> k) & 1u) {
            skip = esc_len(w, wi0 + k, lim) - 1;
        }
    }
    return (uint32_t)skip;
}

// The skip carried into every lane of a step (escapes crossing lanes), from
// `carry` into lane 0: iterated to a fixed point (a chain of lane-crossing
// escapes takes one round per lane it spans; text needs one or two).
__device__ __forceinline__ int lane_skip_in(const uint8_t *w, int wi0, uint32_t ct, uint32_t b, int lim,
                                            uint32_t carry) {
    const int lane = lane_id();
    uint32_t in = lane == 0 ? carry : 0u;
    for (;;) {
        const uint32_t so = lane_spill(w, wi0, ct, b, lim, (int)in);
        uint32_t ni = wave_prev(so);
        if (lane == 0) ni = carry;
        if (!__any(ni != in)) break;
        in = ni;
    }
    return (int)in;
}

__global__ __launch_bounds__(64) void k_json_parse_long(const uint8_t *__restrict__ buf, int64_t len,
                                                        const uint32_t *__restrict__ nl, uint32_t n_nl,
                                                        int64_t n_lines, uint32_t *__restrict__ out_len,
                                                        uint32_t *__restrict__ is_rec, uint2 *__restrict__ span,
                                                        uint32_t *__restrict__ n_invalid) {
    __shared__ __attribute__((aligned(16))) uint8_t s_win[JW_WIN + 16];
    __shared__ uint16_t s_tpos[CHUNK];
    __shared__ uint32_t s_td[CHUNK];
    const int lane = lane_id();
    for (int64_t li = blockIdx.x; li < n_lines; li += gridDim.x) {
        int64_t s, e;
        line_span(nl, n_nl, len, li, &s, &e);
        if (e - s < JL_MIN) continue;
        const int64_t A = s & ~(int64_t)15;
        // carried across steps
        uint32_t esc_par = 0, str_par = 0, D = 0, spill = 0;  // spill: bytes of the next step an escape consumes
        bool bad = false;
        // the grammar walker (lane 0)
        uint64_t stk0 = 0, stk1 = 0;
        int depth = 0, mode = M_VALUE, sub = 0;  // sub: 0 none, 1 value string, 2 key string, 3 number, 4 literal
        bool key_text = false, member_text = false, found = false, ok = true;
        uint32_t f_len = 0, f_s = 0, f_e = 0, str_d0 = 0, nstate = 0;
        int64_t str_s = 0, last_pos = -2;
        const char *lit = nullptr;
        int lit_k = 0;
        uint4 prev = make_uint4(0, 0, 0, 0);  // lane 63: the previous step's last 16 bytes
        for (int64_t b0 = A; b0 < e; b0 += CHUNK) {
            const int64_t p0 = b0 + 16 * lane;
            const uint4 x = p0 < e ? *reinterpret_cast<const uint4 *>(buf + p0) : make_uint4(0, 0, 0, 0);
            const int64_t pn = b0 + CHUNK;
            uint4 nxt = make_uint4(0, 0, 0, 0);
            if (lane == 0 && pn < e) nxt = *reinterpret_cast<const uint4 *>(buf + pn);
            const uint4 pv = make_uint4(lane_bcast(prev.x, 63), lane_bcast(prev.y, 63), lane_bcast(prev.z, 63),
                                        lane_bcast(prev.w, 63));
            __syncthreads();  // the previous step's readers are done with the window and lists
            *reinterpret_cast<uint4 *>(s_win + JW_PRE + 16 * lane) = x;
            if (lane == 0) {
                *reinterpret_cast<uint4 *>(s_win) = pv;
                *reinterpret_cast<uint4 *>(s_win + JW_PRE + CHUNK) = nxt;
            }
            prev = x;
            __syncthreads();
            const JMask m = jmask(x, p0, s, e);
            // escapes
            uint32_t E;
            const uint32_t par_in = esc_carry_in(m.b, m.v, esc_par);
            const uint32_t par_out = esc_mask(m.b, m.v, par_in, &E);
            esc_par = lane_bcast(par_out, 63);
            const uint32_t uq = m.q & ~E;
            // in-string mask: bit k = inside a string just before byte k
            const uint32_t sp = wave_excl_xor((uint32_t)__builtin_popcount(uq) & 1u) ^ str_par;
            uint32_t ins = 0, par = sp;
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                ins |= par << k;
                par ^= (uq >> k) & 1u;
            }
            str_par = lane_bcast(par, 63);
            const uint32_t ct = ins & ~uq & m.v;  // string content bytes
            const int lim = (int)((e - b0) < (int64_t)(CHUNK + 16) ? (e - b0) : (int64_t)(CHUNK + 16)) + JW_PRE;
            const uint8_t *w = s_win;
            // content checks and decoded lengths; an escape may consume bytes of the
            // next lane (or step)
            const int wi0 = JW_PRE + 16 * lane;
            int skip = lane_skip_in(w, wi0, ct, m.b, lim, spill);
            uint32_t dsum = 0;
            uint32_t dl_pre[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const int wi = wi0 + k;
                uint32_t dl = 0;
                if (skip > 0) {
                    --skip;  // inside an escape sequence
                } else if ((ct >> k) & 1u) {
                    const uint32_t c = w[wi];
                    if ((m.b >> k) & 1u) {
                        int d = 1;
                        uint32_t cp;
                        skip = esc_info(w, wi, lim, &d, &cp, &bad) - 1;
                        dl = (uint32_t)d;
                    } else if (c < 0x20u) {
                        bad = true;
                    } else if (c >= 0x80u) {
                        if ((c & 0xC0u) == 0x80u) {
                            // continuation: the nearest non-continuation byte before must cover it
                            int q = wi - 1, back = 1;
                            while (back < 4 && (w[q] & 0xC0u) == 0x80u) { --q; ++back; }
                            const uint32_t ld = w[q];
                            const int l = (ld & 0xE0u) == 0xC0u ? 2 : (ld & 0xF0u) == 0xE0u ? 3 : (ld & 0xF8u) == 0xF0u ? 4 : 0;
                            if (l <= back) bad = true;
                        } else {
                            int l;
                            uint32_t cp, mn;
                            if ((c & 0xE0u) == 0xC0u) { l = 2; cp = c & 0x1Fu; mn = 0x80u; }
                            else if ((c & 0xF0u) == 0xE0u) { l = 3; cp = c & 0x0Fu; mn = 0x800u; }
                            else if ((c & 0xF8u) == 0xF0u) { l = 4; cp = c & 0x07u; mn = 0x10000u; }
                            else { l = 1; cp = 0; mn = 1; bad = true; }
                            if (wi + l > lim) bad = true;
                            for (int t = 1; t < l && wi + t < lim; ++t) {
                                const uint32_t y = w[wi + t];
                                if ((y & 0xC0u) != 0x80u) bad = true;
                                cp = cp << 6 | (y & 0x3Fu);
                            }
                            if (cp < mn || cp > 0x10FFFFu || (cp >= 0xD800u && cp <= 0xDFFFu)) bad = true;
                        }
                        dl = 1;
                    } else {
                        dl = 1;
                    }
                }
                dl_pre[k] = dsum;
                dsum += dl;
            }
            spill = lane_bcast((uint32_t)skip, 63);  // into the next step's lane 0
            // decoded-length prefix at every byte
            const uint32_t dex = wave_incl_sum(dsum) - dsum + D;
            D = lane_bcast(dex + dsum, 63);
            // tokens: quotes and non-ws bytes outside strings
            const uint32_t tk = m.v & (uq | (~ins & ~m.w));
            const uint32_t nt_l = (uint32_t)__builtin_popcount(tk);
            const uint32_t tb = wave_incl_sum(nt_l) - nt_l;
            const uint32_t ntok = lane_bcast(tb + nt_l, 63);
            {
                uint32_t at = tb;
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    if ((tk >> k) & 1u) {
                        s_tpos[at] = (uint16_t)(16 * lane + k);
                        s_td[at] = dex + dl_pre[k];
                        ++at;
                    }
            }
            __syncthreads();
            // the grammar over this step's tokens (lane 0)
            if (lane == 0 && ok) {
                for (uint32_t t = 0; t < ntok && ok; ++t) {
                    const int64_t pos = b0 + s_tpos[t];
                    const uint32_t c = w[JW_PRE + s_tpos[t]];
                    const uint32_t dpre = s_td[t];
                    bool again = true;
                    while (again && ok) {
                        again = false;
                        if (sub == 1 || sub == 2) {  // the closing quote of the current string
                            if (sub == 1) {
                                if (member_text) {
                                    found = true;
                                    f_len = dpre - str_d0;
                                    f_s = (uint32_t)str_s;
                                    f_e = (uint32_t)pos;
                                }
                                mode = M_AFTER;
                            } else {
                                // key: "text" at depth 1 (escapes decoded; keys are short)
                                bool is_text = false;
                                if (depth == 1 && dpre - str_d0 == 4u) {
                                    LaneReader rd{buf, -1, make_uint4(0, 0, 0, 0)};
                                    int64_t q = str_s;
                                    uint32_t n;
                                    is_text = json_string(rd, q, e, &n, true, &is_text) && is_text;
                                }
                                key_text = is_text;
                                mode = M_KEY + 10;  // expecting ':'
                            }
                            sub = 0;
                            break;
                        }
                        if (sub == 3) {  // number continues while consecutive number chars fit the grammar
                            const bool adj = pos == last_pos + 1;
                            bool take = false;
                            if (adj) {
                                const bool dg = c - '0' < 10u;
                                switch (nstate) {
                                    case 0: take = dg; if (dg) nstate = c == '0' ? 1 : 2; break;            // after '-'
                                    case 1: take = c == '.' || (c | 0x20u) == 'e'; break;                     // after leading 0
                                    case 2: take = dg || c == '.' || (c | 0x20u) == 'e'; break;               // int digits
                                    case 3: take = dg; if (dg) nstate = 4; break;                             // after '.'
                                    case 4: take = dg || (c | 0x20u) == 'e'; break;                           // frac digits
                                    case 5: take = dg || c == '+' || c == '-'; if (take) nstate = dg ? 7 : 6; break;  // after e
                                    case 6: take = dg; if (dg) nstate = 7; break;                             // after e sign
                                    case 7: take = dg; break;                                                 // exp digits
                                }
                                if (take && (nstate == 1 || nstate == 2) && c == '.') nstate = 3;
                                else if (take && (nstate == 1 || nstate == 2 || nstate == 4) && (c | 0x20u) == 'e') nstate = 5;
                            }
                            if (take) { last_pos = pos; break; }
                            if (!(nstate == 1 || nstate == 2 || nstate == 4 || nstate == 7)) { ok = false; break; }
                            sub = 0;
                            mode = M_AFTER;
                            again = true;  // this token follows the number
                            continue;
                        }
                        if (sub == 4) {  // literal continues
                            if (pos != last_pos + 1 || c != (uint32_t)lit[lit_k]) { ok = false; break; }
                            last_pos = pos;
                            if (!lit[++lit_k]) { sub = 0; mode = M_AFTER; }
                            break;
                        }
                        if (mode == M_KEY + 10) {  // ':' after a key
                            if (c != ':') { ok = false; break; }
                            mode = M_VALUE;
                            break;
                        }
                        if (mode == M_AFTER && depth == 0) { ok = false; break; }  // trailing characters
                        if (mode == M_VALUE) {
                            member_text = key_text;
                            key_text = false;
                            if (c == '{' || c == '[') {
                                if (depth >= JSON_MAX_DEPTH) { ok = false; break; }
                                const uint64_t bit = c == '{' ? 1ull : 0ull;
                                if (depth < 64) stk0 = (stk0 & ~(1ull << depth)) | (bit << depth);
                                else stk1 = (stk1 & ~(1ull << (depth - 64))) | (bit << (depth - 64));
                                ++depth;
                                if (member_text) found = false;
                                mode = c == '{' ? M_KEY + 20 : M_VALUE + 20;  // first member / element or the closer
                                break;
                            }
                            if (c == '"') { sub = 1; str_s = pos + 1; str_d0 = dpre; break; }
                            if (member_text) found = false;
                            if (c == '-' || c - '0' < 10u) {
                                sub = 3;
                                nstate = c == '-' ? 0 : c == '0' ? 1 : 2;
                                last_pos = pos;
                                break;
                            }
                            lit = c == 't' ? "true" : c == 'f' ? "false" : c == 'n' ? "null" : nullptr;
                            if (!lit) { ok = false; break; }
                            sub = 4;
                            lit_k = 1;
                            last_pos = pos;
                            break;
                        }
                        if (mode == M_KEY + 20 || mode == M_VALUE + 20) {  // just opened: the closer or the first item
                            const bool obj = mode == M_KEY + 20;
                            if (c == (obj ? '}' : ']')) { --depth; mode = M_AFTER; break; }
                            mode = obj ? M_KEY : M_VALUE;
                            again = true;
                            continue;
                        }
                        if (mode == M_KEY) {
                            if (c != '"') { ok = false; break; }
                            sub = 2;
                            str_s = pos + 1;
                            str_d0 = dpre;
                            break;
                        }
                        // M_AFTER inside a container
                        const int b = depth - 1;
                        const bool obj = b < 64 ? (stk0 >> b) & 1ull : (stk1 >> (b - 64)) & 1ull;
                        if (c == ',') { mode = obj ? M_KEY : M_VALUE; break; }
                        if (c == (obj ? '}' : ']')) { --depth; mode = M_AFTER; break; }
                        ok = false;
                    }
                }
            }
            __syncthreads();
        }
        // end of line: a number may end it; anything else open is an error
        const uint64_t bad_lanes = __ballot(bad);
        if (lane == 0) {
            if (ok && sub == 3) {
                if (nstate == 1 || nstate == 2 || nstate == 4 || nstate == 7) { sub = 0; mode = M_AFTER; }
                else ok = false;
            }
            if (sub != 0 || str_par) ok = false;
            ok = ok && bad_lanes == 0 && mode == M_AFTER && depth == 0;
            const bool rec = ok && found;
            out_len[li] = rec ? f_len : 0u;
            is_rec[li] = rec ? 1u : 0u;
            span[li] = make_uint2(f_s, f_e);
            if (!ok) atomicAdd(n_invalid, 1u);
        }
    }
}

// Decode of long record lines: one wave per line, 1 KiB of the string per step.
__global__ __launch_bounds__(64) void k_json_write_long(const uint8_t *__restrict__ buf, const uint32_t *__restrict__ nl,
                                                        uint32_t n_nl, int64_t len, int64_t n_lines,
                                                        const uint32_t *__restrict__ is_rec,
                                                        const uint2 *__restrict__ span,
                                                        const uint32_t *__restrict__ toff,
                                                        uint8_t *__restrict__ text) {
    __shared__ __attribute__((aligned(16))) uint8_t s_win[JW_WIN + 16];
    const int lane = lane_id();
    for (int64_t li = blockIdx.x; li < n_lines; li += gridDim.x) {
        int64_t ls, le;
        line_span(nl, n_nl, len, li, &ls, &le);
        if (le - ls < JL_MIN || !is_rec[li]) continue;
        const int64_t s = span[li].x, e = span[li].y;
        const int64_t A = s & ~(int64_t)15;
        uint32_t esc_par = 0, spill = 0;
        uint8_t *o = text + toff[li];
        uint32_t O = 0;  // output bytes written so far
        for (int64_t b0 = A; b0 < e; b0 += CHUNK) {
            const int64_t p0 = b0 + 16 * lane;
            const uint4 x = p0 < e ? *reinterpret_cast<const uint4 *>(buf + p0) : make_uint4(0, 0, 0, 0);
            uint4 nxt = make_uint4(0, 0, 0, 0);
            if (lane == 0 && b0 + CHUNK < e) nxt = *reinterpret_cast<const uint4 *>(buf + b0 + CHUNK);
            __syncthreads();
            *reinterpret_cast<uint4 *>(s_win + JW_PRE + 16 * lane) = x;
            if (lane == 0) *reinterpret_cast<uint4 *>(s_win + JW_PRE + CHUNK) = nxt;
            __syncthreads();
            const JMask m = jmask(x, p0, s, e);
            uint32_t E;
            const uint32_t par_in = esc_carry_in(m.b, m.v, esc_par);
            const uint32_t par_out = esc_mask(m.b, m.v, par_in, &E);
            esc_par = lane_bcast(par_out, 63);
            const int lim = (int)((e - b0) < (int64_t)(CHUNK + 16) ? (e - b0) : (int64_t)(CHUNK + 16)) + JW_PRE;
            const uint8_t *w = s_win;
            const int wi0 = JW_PRE + 16 * lane;
            const int skip = lane_skip_in(w, wi0, m.v, m.b, lim, spill);
            // pass 1: output length of this lane's bytes
            uint32_t cnt = 0;
            int sk_end;
            {
                int sk = skip;
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    if (sk > 0) {
                        --sk;
                    } else if ((m.v >> k) & 1u) {
                        if ((m.b >> k) & 1u) {
                            int d = 1;
                            uint32_t cp;
                            bool bad = false;
                            sk = esc_info(w, wi0 + k, lim, &d, &cp, &bad) - 1;
                            cnt += (uint32_t)d;
                        } else {
                            cnt += 1;
                        }
                    }
                }
                sk_end = sk;
            }
            const uint32_t at = wave_incl_sum(cnt) - cnt + O;
            O = lane_bcast(at + cnt, 63);
            const uint32_t sp_last = lane_bcast((uint32_t)sk_end, 63);
            // pass 2: write
            {
                uint32_t q = at;
                int sk = skip;
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const int wi = wi0 + k;
                    if (sk > 0) {
                        --sk;
                    } else if ((m.v >> k) & 1u) {
                        if ((m.b >> k) & 1u) {
                            int d = 1;
                            uint32_t cp;
                            bool bad = false;
                            sk = esc_info(w, wi, lim, &d, &cp, &bad) - 1;
                            if (cp < 0x80u) {
                                o[q++] = (uint8_t)cp;
                            } else if (cp < 0x800u) {
                                o[q++] = (uint8_t)(0xC0u | cp >> 6);
                                o[q++] = (uint8_t)(0x80u | (cp & 0x3Fu));
                            } else if (cp < 0x10000u) {
                                o[q++] = (uint8_t)(0xE0u | cp >> 12);
                                o[q++] = (uint8_t)(0x80u | ((cp >> 6) & 0x3Fu));
                                o[q++] = (uint8_t)(0x80u | (cp & 0x3Fu));
                            } else {
                                o[q++] = (uint8_t)(0xF0u | cp >> 18);
                                o[q++] = (uint8_t)(0x80u | ((cp >> 12) & 0x3Fu));
                                o[q++] = (uint8_t)(0x80u | ((cp >> 6) & 0x3Fu));
                                o[q++] = (uint8_t)(0x80u | (cp & 0x3Fu));
                            }
                        } else {
                            o[q++] = w[wi];
                        }
                    }
                }
            }
            // the next step's lane 0 continues lane 63's escape
            spill = sp_last;
        }
    }
}

hipError_t launch_json_nl_count(const uint8_t *buf, int64_t len, uint32_t *cnt, uint32_t *base, uint32_t *scan_tmp,
                                hipStream_t st) {
    const int64_t nb = (len + CHUNK - 1) / CHUNK;
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(k_json_nl_count, dim3((unsigned)nb), dim3(64), 0, st, buf, len, cnt);
    return launch_exclusive_scan(cnt, base, nb, scan_tmp, st);
}

hipError_t launch_json_nl_write(const uint8_t *buf, int64_t len, const uint32_t *base, uint32_t *nl, uint32_t cap,
                                hipStream_t st) {
    const int64_t nb = (len + CHUNK - 1) / CHUNK;
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(k_json_nl_write, dim3((unsigned)nb), dim3(64), 0, st, buf, len, base, nl, cap);
    return hipGetLastError();
}

// {newline count, position of the last newline} in one word pair, so the host
// reads both with one copy and one synchronisation
// (the position is only valid when the list held every newline, n <= cap)
__global__ void k_json_nl_tail(const uint32_t *__restrict__ total, const uint32_t *__restrict__ nl, uint32_t cap,
                               uint32_t *__restrict__ out) {
    const uint32_t n = *total;
    out[0] = n;
    out[1] = n && n <= cap ? nl[n - 1] : 0u;
}

hipError_t launch_json_nl_tail(const uint32_t *total, const uint32_t *nl, uint32_t cap, uint32_t *out, hipStream_t st) {
    hipLaunchKernelGGL(k_json_nl_tail, dim3(1), dim3(1), 0, st, total, nl, cap, out);
    return hipGetLastError();
}

hipError_t launch_json_parse(const uint8_t *buf, int64_t len, const uint32_t *nl, uint32_t n_nl, int64_t n_lines,
                             uint32_t *out_len, uint32_t *is_rec, uint2 *span, uint32_t *n_invalid, hipStream_t st) {
    if (n_lines == 0) return hipSuccess;
    hipLaunchKernelGGL(k_json_parse, dim3((unsigned)((n_lines + 255) / 256)), dim3(256), 0, st, buf, len, nl, n_nl,
                       n_lines, out_len, is_rec, span, n_invalid);
    // lines >= JL_MIN bytes: one wave each (persistent grid over the line list)
    const int64_t waves = n_lines < 8192 ? n_lines : 8192;
    hipLaunchKernelGGL(k_json_parse_long, dim3((unsigned)waves), dim3(64), 0, st, buf, len, nl, n_nl, n_lines, out_len,
                       is_rec, span, n_invalid);
    return hipGetLastError();
}

hipError_t launch_json_write(const uint8_t *buf, int64_t len, const uint32_t *nl, uint32_t n_nl, int64_t n_lines,
                             const uint32_t *is_rec, const uint2 *span, const uint32_t *toff, const uint32_t *ridx,
                             uint8_t *text, uint64_t *offsets, hipStream_t st) {
    if (n_lines == 0) return hipSuccess;
    hipLaunchKernelGGL(k_json_write, dim3((unsigned)((n_lines + 255) / 256)), dim3(256), 0, st, buf, nl, n_nl, len,
                       n_lines, is_rec, span, toff, ridx, text, offsets);
    const int64_t waves = n_lines < 8192 ? n_lines : 8192;
    hipLaunchKernelGGL(k_json_write_long, dim3((unsigned)waves), dim3(64), 0, st, buf, nl, n_nl, len, n_lines, is_rec,
                       span, toff, text);
    return hipGetLastError();
}

}  // namespace sdl
