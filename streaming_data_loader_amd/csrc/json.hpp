// json.hpp -- minimal JSON reader for HF tokenizer.json assets.
//
// The reference obtains its tokenizer with Tokenizer::from_pretrained(name)
// (rust/src/tokenizer/tokenizer_holder.rs:64-82), i.e. a tokenizer.json from
// the hub.  This reader parses the same file format (objects, arrays, strings
// with \uXXXX escapes incl. surrogate pairs, numbers, true/false/null) into a
// small tree; only what the Batcher needs is then read from it.
#pragma once

#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace sdl {

struct JValue {
    enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
    bool b = false;
    double num = 0.0;
    std::string str;
    std::vector<JValue> arr;
    std::vector<std::pair<std::string, JValue>> obj;  // file order preserved

    const JValue *get(const std::string &k) const {
        if (kind != OBJ) return nullptr;
        for (auto &kv : obj)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
    bool is_str(const char *s) const { return kind == STR && str == s; }
};

class JParser {
   public:
    explicit JParser(const std::string &s) : s_(s) {}
    JValue parse() {
        JValue v = value();
        ws();
        if (i_ != s_.size()) fail("trailing data");
        return v;
    }

   private:
    const std::string &s_;
    size_t i_ = 0;

    [[noreturn]] void fail(const char *m) { throw std::runtime_error(std::string("json: ") + m + " at " + std::to_string(i_)); }
    void ws() {
        while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\r' || s_[i_] == '\t')) ++i_;
    }
    char peek() {
        ws();
        if (i_ >= s_.size()) fail("eof");
        return s_[i_];
    }
    void expect(char c) {
        if (peek() != c) fail("unexpected char");
        ++i_;
    }
    static void put_utf8(std::string &o, uint32_t cp) {
        if (cp < 0x80) o += (char)cp;
        else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
        else if (cp < 0x10000) { o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
        else { o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
    }
    uint32_t hex4() {
        if (i_ + 4 > s_.size()) fail("short \\u");
        uint32_t v = 0;
        for (int k = 0; k < 4; ++k) {
            char c = s_[i_++];
            v <<= 4;
            if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
            else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
            else fail("bad hex");
        }
        return v;
    }
    std::string string() {
        expect('"');
        std::string o;
        while (true) {
            if (i_ >= s_.size()) fail("eof in string");
            char c = s_[i_++];
            if (c == '"') break;
            if (c != '\\') { o += c; continue; }
            char e = s_[i_++];
            switch (e) {
                case '"': o += '"'; break;
                case '\\': o += '\\'; break;
                case '/': o += '/'; break;
                case 'b': o += '\b'; break;
                case 'f': o += '\f'; break;
                case 'n': o += '\n'; break;
                case 'r': o += '\r'; break;
                case 't': o += '\t'; break;
                case 'u': {
                    uint32_t cp = hex4();
                    if (cp >= 0xD800 && cp < 0xDC00 && i_ + 6 <= s_.size() && s_[i_] == '\\' && s_[i_ + 1] == 'u') {
                        i_ += 2;
                        uint32_t lo = hex4();
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                    }
                    put_utf8(o, cp);
                    break;
                }
                default: fail("bad escape");
            }
        }
        return o;
    }
    JValue value() {
        char c = peek();
        JValue v;
        if (c == '{') {
            ++i_;
            v.kind = JValue::OBJ;
            if (peek() == '}') { ++i_; return v; }
            while (true) {
                std::string k = string();
                expect(':');
                v.obj.emplace_back(std::move(k), value());
                char d = peek();
                ++i_;
                if (d == '}') break;
                if (d != ',') fail("expected , or }");
            }
        } else if (c == '[') {
            ++i_;
            v.kind = JValue::ARR;
            if (peek() == ']') { ++i_; return v; }
            while (true) {
                v.arr.push_back(value());
                char d = peek();
                ++i_;
                if (d == ']') break;
                if (d != ',') fail("expected , or ]");
            }
        } else if (c == '"') {
            v.kind = JValue::STR;
            v.str = string();
        } else if (s_.compare(i_, 4, "true") == 0) {
            i_ += 4; v.kind = JValue::BOOL; v.b = true;
        } else if (s_.compare(i_, 5, "false") == 0) {
            i_ += 5; v.kind = JValue::BOOL;
        } else if (s_.compare(i_, 4, "null") == 0) {
            i_ += 4;
        } else {
            v.kind = JValue::NUM;
            v.num = number();
        }
        return v;
    }

    // A number read the way serde_json (1.0.87 in the reference's Cargo.lock,
    // default features, no `float_roundtrip`) reads it into the f64 that
    // tokenizers' Unigram keeps as a piece score: the digits go into a u64
    // mantissa until one more would overflow it (then integer digits only
    // scale, fraction digits are ignored), and the result is
    // (double)mantissa * or / the correctly rounded power of ten -- not the
    // correctly rounded value strtod gives.  The difference (an ulp for ~1/4
    // of 17-digit scores) decides Viterbi ties between equal-sum paths.
    double number() {
        static const std::vector<double> p10 = [] {
            std::vector<double> t(309);
            for (int k = 0; k < 309; ++k) t[(size_t)k] = std::strtod(("1e" + std::to_string(k)).c_str(), nullptr);
            return t;
        }();
        auto digit = [&]() -> int {
            return i_ < s_.size() && s_[i_] >= '0' && s_[i_] <= '9' ? s_[i_] - '0' : -1;
        };
        const bool neg = i_ < s_.size() && s_[i_] == '-';
        if (neg) ++i_;
        if (digit() < 0) fail("bad value");
        uint64_t m = 0;
        int64_t e10 = 0;
        bool full = false;  // the mantissa took its last digit
        auto take = [&](int d, bool fraction) {
            if (!full && (m > UINT64_MAX / 10 || (m == UINT64_MAX / 10 && (uint64_t)d > UINT64_MAX % 10))) full = true;
            if (full) {
                if (!fraction) ++e10;
                return;
            }
            m = m * 10 + (uint64_t)d;
            if (fraction) --e10;
        };
        if (digit() == 0) {
            ++i_;
            if (digit() >= 0) fail("leading zero");
        } else {
            for (int d; (d = digit()) >= 0; ++i_) take(d, false);
        }
        if (i_ < s_.size() && s_[i_] == '.') {
            ++i_;
            if (digit() < 0) fail("bad fraction");
            // (after an integer-part overflow serde_json retries each fraction
            // digit against the same u64 bound, as `take` does)
            full = false;
            for (int d; (d = digit()) >= 0; ++i_) take(d, true);
        }
        if (i_ < s_.size() && (s_[i_] == 'e' || s_[i_] == 'E')) {
            ++i_;
            bool eneg = false;
            if (i_ < s_.size() && (s_[i_] == '+' || s_[i_] == '-')) eneg = s_[i_++] == '-';
            if (digit() < 0) fail("bad exponent");
            int64_t x = 0;
            bool big = false;
            for (int d; (d = digit()) >= 0; ++i_) {
                if (x > INT32_MAX / 10 || (x == INT32_MAX / 10 && d > INT32_MAX % 10)) big = true;
                if (!big) x = x * 10 + d;
            }
            if (big) {
                if (m != 0 && !eneg) fail("number out of range");
                return neg ? -0.0 : 0.0;
            }
            e10 = eneg ? e10 - x : e10 + x;
            e10 = e10 > INT32_MAX ? INT32_MAX : e10 < INT32_MIN ? INT32_MIN : e10;
        }
        double f = (double)m;
        while (true) {
            const int64_t a = e10 < 0 ? -e10 : e10;
            if (a <= 308) {
                if (e10 >= 0) {
                    f *= p10[(size_t)a];
                    if (f > 1.7976931348623157e308) fail("number out of range");
                } else {
                    f /= p10[(size_t)a];
                }
                break;
            }
            if (f == 0.0) break;
            if (e10 >= 0) fail("number out of range");
            f /= 1e308;
            e10 += 308;
        }
        return neg ? -f : f;
    }
};

}  // namespace sdl
