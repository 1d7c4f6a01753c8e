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
            const char *b = s_.c_str() + i_;
            char *e = nullptr;
            v.kind = JValue::NUM;
            v.num = std::strtod(b, &e);
            if (e == b) fail("bad value");
            i_ += (size_t)(e - b);
        }
        return v;
    }
};

}  // namespace sdl
