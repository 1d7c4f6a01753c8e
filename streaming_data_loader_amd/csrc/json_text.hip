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
                                                      const uint32_t *__restrict__ base, uint32_t *__restrict__ nl) {
    const int64_t p0 = (int64_t)blockIdx.x * CHUNK + 16 * threadIdx.x;
    uint32_t m = 0;
    if (p0 < len) {
        const uint4 v = *reinterpret_cast<const uint4 *>(buf + p0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        for (int i = 0; i < 16 && p0 + i < len; ++i) m |= (((w[i >> 2] >> (8 * (i & 3))) & 0xFFu) == '\n' ? 1u : 0u) << i;
    }
    const uint32_t c = (uint32_t)__builtin_popcount(m);
    uint32_t at = base[blockIdx.x] + wave_incl_sum(c) - c;
    for (; m; m &= m - 1) nl[at++] = (uint32_t)(p0 + __builtin_ctz(m));
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
__global__ __launch_bounds__(256) void k_json_write(const uint8_t *__restrict__ buf, int64_t n_lines,
                                                    const uint32_t *__restrict__ is_rec, const uint2 *__restrict__ span,
                                                    const uint32_t *__restrict__ toff, const uint32_t *__restrict__ ridx,
                                                    uint8_t *__restrict__ text, uint64_t *__restrict__ offsets) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_lines) return;
    if (i == n_lines - 1) offsets[ridx[n_lines]] = toff[n_lines];  // offsets[n_records] = total bytes
    if (!is_rec[i]) return;
    offsets[ridx[i]] = toff[i];
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

hipError_t launch_json_nl_count(const uint8_t *buf, int64_t len, uint32_t *cnt, uint32_t *base, uint32_t *scan_tmp,
                                hipStream_t st) {
    const int64_t nb = (len + CHUNK - 1) / CHUNK;
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(k_json_nl_count, dim3((unsigned)nb), dim3(64), 0, st, buf, len, cnt);
    return launch_exclusive_scan(cnt, base, nb, scan_tmp, st);
}

hipError_t launch_json_nl_write(const uint8_t *buf, int64_t len, const uint32_t *base, uint32_t *nl, hipStream_t st) {
    const int64_t nb = (len + CHUNK - 1) / CHUNK;
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(k_json_nl_write, dim3((unsigned)nb), dim3(64), 0, st, buf, len, base, nl);
    return hipGetLastError();
}

hipError_t launch_json_parse(const uint8_t *buf, int64_t len, const uint32_t *nl, uint32_t n_nl, int64_t n_lines,
                             uint32_t *out_len, uint32_t *is_rec, uint2 *span, uint32_t *n_invalid, hipStream_t st) {
    if (n_lines == 0) return hipSuccess;
    hipLaunchKernelGGL(k_json_parse, dim3((unsigned)((n_lines + 255) / 256)), dim3(256), 0, st, buf, len, nl, n_nl,
                       n_lines, out_len, is_rec, span, n_invalid);
    return hipGetLastError();
}

hipError_t launch_json_write(const uint8_t *buf, int64_t n_lines, const uint32_t *is_rec, const uint2 *span,
                             const uint32_t *toff, const uint32_t *ridx, uint8_t *text, uint64_t *offsets,
                             hipStream_t st) {
    if (n_lines == 0) return hipSuccess;
    hipLaunchKernelGGL(k_json_write, dim3((unsigned)((n_lines + 255) / 256)), dim3(256), 0, st, buf, n_lines, is_rec,
                       span, toff, ridx, text, offsets);
    return hipGetLastError();
}

}  // namespace sdl
