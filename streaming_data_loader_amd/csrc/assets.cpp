// assets.cpp -- loads the tokenizer the Batcher runs (tokenizer_holder.rs:64-97
// gets it from the HF hub with Tokenizer::from_pretrained; here the same
// tokenizer.json format is read from disk) and packs it for the device.
#include "assets.hpp"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <array>
#include <cstdio>
#include <queue>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <unordered_set>
#include <unordered_map>
#include <unordered_set>

#include "json.hpp"
#include "unigram.hpp"

namespace sdl {

uint32_t piece_hash(const uint8_t *payload, size_t n, uint32_t cont) {
    uint32_t h = ph_init((uint32_t)n, cont);
    size_t b0 = 0;
    do {  // at least one block, even for an empty payload
        uint32_t w[4] = {0, 0, 0, 0};
        for (size_t k = 0; k < 16 && b0 + k < n; ++k) w[k >> 2] |= (uint32_t)payload[b0 + k] << (8 * (k & 3));
        for (int i = 0; i < 4; ++i) h = ph_mix(h, w[i]);
        b0 += 16;
    } while (b0 < n);
    return ph_final(h);
}

static std::string read_file(const std::string &path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open " + path);
    std::ostringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

static void load_unicode(const std::string &path, HostTokenizer &t) {
    std::string d = read_file(path);
    if (d.size() < 20 || std::memcmp(d.data(), "SDLU", 4) != 0) throw std::runtime_error("bad unicode table " + path);
    uint32_t hdr[4];
    std::memcpy(hdr, d.data() + 4, 16);
    if (hdr[0] != 2) throw std::runtime_error("unicode table version mismatch (tools/make_unicode_tables.py)");
    const size_t np = hdr[1], nb = hdr[2], pb = hdr[3];
    if (np != 0x110000 / 128 || d.size() != 20 + 2 * np + 4 * 128 * nb + pb)
        throw std::runtime_error("unicode table size mismatch");
    t.upage.resize(np);
    t.uentry.resize(128 * nb);
    t.upool.resize(pb + 16);
    std::memcpy(t.upage.data(), d.data() + 20, 2 * np);
    std::memcpy(t.uentry.data(), d.data() + 20 + 2 * np, 4 * 128 * nb);
    std::memcpy(t.upool.data(), d.data() + 20 + 2 * np + 4 * 128 * nb, pb);
    // The kernels' ASCII fast path lower-cases A-Z itself: check the table agrees.
    for (uint32_t c = 0; c < 128; ++c) {
        uint32_t e = t.uentry[(size_t)t.upage[0] * 128 + c];
        if ((e & 3u) != UC_OTHER) continue;
        uint8_t want = (uint8_t)((c - 'A' < 26u) ? c + 32 : c);
        uint8_t got = (e & 4u) ? (uint8_t)c : t.upool[(e >> 8) + 2];
        if (got != want || (!(e & 4u) && t.upool[e >> 8] != 1))
            throw std::runtime_error("unicode table: unexpected ASCII mapping");
    }
}

static bool is_bert_normalizer(const JValue *n) {
    if (!n) return false;
    const JValue *t = n->get("type");
    if (!t || !t->is_str("BertNormalizer")) return false;
    auto flag = [&](const char *k, bool dflt) {
        const JValue *v = n->get(k);
        return (v && v->kind == JValue::BOOL) ? v->b : dflt;
    };
    const JValue *sa = n->get("strip_accents");
    bool strip = (sa && sa->kind == JValue::BOOL) ? sa->b : flag("lowercase", true);
    return flag("clean_text", true) && flag("handle_chinese_chars", true) && flag("lowercase", true) && strip;
}

static int find_piece(const HostTokenizer &t, const std::string &s) {
    for (size_t i = t.pieces.size(); i-- > 0;)
        if (t.pieces[i] == s) return (int)i;  // a duplicated piece keeps its last id (HashMap insert)
    return -1;
}

static bool cuckoo_insert(std::vector<VSlot> &tab, uint32_t mask, VSlot v) {
    uint32_t pos = cuckoo_slot1(v.hash, mask);
    for (int kick = 0; kick < 2000; ++kick) {
        if (tab[pos].id < 0) {
            tab[pos] = v;
            return true;
        }
        std::swap(v, tab[pos]);  // evict the occupant to its other slot
        const uint32_t a = cuckoo_slot1(v.hash, mask), b = cuckoo_slot2(v.hash, mask);
        pos = pos == a ? b : a;
    }
    return false;
}

static void build_vocab_table(HostTokenizer &t) {
    const size_t n = t.pieces.size();
    if (n > 65535) throw std::runtime_error("vocabulary larger than 65535 ids is not supported (u16 staging)");
    std::unordered_map<std::string, int> last;  // HF vocab is a map: duplicates keep the last id
    for (size_t id = 0; id < n; ++id) last[t.pieces[id]] = (int)id;
    std::vector<VSlot> entries;
    t.vpool.clear();
    t.maxlen_first = t.maxlen_cont = 0;
    t.wp_lens[0].clear();
    t.wp_lens[1].clear();
    t.wp_long_pieces = false;
    for (size_t id = 0; id < n; ++id) {
        const std::string &s = t.pieces[id];
        if (s.empty() || last[s] != (int)id) continue;
        const uint32_t cont = (s.size() > 2 && s[0] == '#' && s[1] == '#') ? 1u : 0u;
        const std::string pay = cont ? s.substr(2) : s;
        if (pay.size() > 255) throw std::runtime_error("vocabulary piece longer than 255 bytes");
        if (cont) t.maxlen_cont = std::max(t.maxlen_cont, (int)pay.size());
        else t.maxlen_first = std::max(t.maxlen_first, (int)pay.size());
        if (pay.size() > (size_t)LW_MAX) t.wp_long_pieces = true;
        else if (std::find(t.wp_lens[cont].begin(), t.wp_lens[cont].end(), (uint8_t)pay.size()) == t.wp_lens[cont].end())
            t.wp_lens[cont].push_back((uint8_t)pay.size());
        VSlot v{};
        v.key = (uint32_t)pay.size() | (cont << 8);
        v.id = (int32_t)id;
        v.pool_off = (uint32_t)t.vpool.size();
        v.hash = piece_hash((const uint8_t *)pay.data(), pay.size(), cont);
        std::memcpy(v.inl, pay.data(), std::min<size_t>(16, pay.size()));
        t.vpool.insert(t.vpool.end(), pay.begin(), pay.end());
        entries.push_back(v);
    }
    t.vpool.resize(t.vpool.size() + 64, 0);
    uint32_t slots = 1;
    while (slots < 4 * entries.size()) slots <<= 1;  // load <= 0.25
    for (;; slots <<= 1) {
        t.slot_mask = slots - 1;
        t.slots.assign(slots, VSlot{0, -1, 0, 0, {0}});
        bool ok = true;
        for (const VSlot &v : entries)
            if (!cuckoo_insert(t.slots, t.slot_mask, v)) { ok = false; break; }
        if (ok) break;
        if (slots >= (1u << 24)) throw std::runtime_error("cuckoo table build failed");
    }
}

// ASCII visible classes the kernels compute arithmetically (tokenize_wordpiece.hip:
// ascii_vclass) must be the table's; and the one-byte ids of the ISO fast path.
static void check_ascii_and_ids(HostTokenizer &t) {
    t.ascii_id.assign(128, t.unk_id);
    for (uint32_t b = 0; b < 128; ++b) {
        const uint32_t e = t.uentry[(size_t)t.upage[0] * 128 + b];
        uint32_t want;
        const uint32_t l = b | 0x20u;
        if (l - 'a' < 26u || b - '0' < 10u) want = UC_OTHER;
        else if (b == ' ' || b == '\t' || b == '\n' || b == '\r') want = UC_WS;
        else if (b < 32u || b == 127u) want = UC_DEL;
        else want = UC_ISO;
        if ((e & 3u) != want) throw std::runtime_error("unicode table: ASCII classes differ from the kernels' classifier");
        std::string m = (e & 4u) ? std::string(1, (char)b)
                                 : std::string((const char *)&t.upool[(e >> 8) + 2], t.upool[e >> 8]);
        const int id = find_piece(t, m);
        if (id >= 0) t.ascii_id[b] = id;
    }
    if (t.opener && (t.opener >= 0x80 || (t.uentry[(size_t)t.upage[0] * 128 + t.opener] & 3u) == UC_OTHER))
        throw std::runtime_error("added tokens must start with an ASCII non-alphanumeric byte");
}

static void set_added(HostTokenizer &t) {
    t.opener = 0;
    t.max_special_len = 0;
    if (t.added.empty()) return;
    if ((int)t.added.size() > MAX_SPECIAL) throw std::runtime_error("too many added tokens");
    const uint8_t op = (uint8_t)t.added[0].first[0];
    for (auto &a : t.added) {
        const std::string &s = a.first;
        if (s.empty() || (int)s.size() > MAX_SPECIAL_LEN) throw std::runtime_error("added token length unsupported");
        if ((uint8_t)s[0] != op || s.find((char)op, 1) != std::string::npos)
            throw std::runtime_error("added tokens must share a first byte that occurs nowhere else in them");
        t.max_special_len = std::max(t.max_special_len, (int)s.size());
    }
    t.opener = op;
}

// Device entry format: the file's entries with short normalizations (<= 3
// bytes) moved inline -- bits 0-1 class, bit 2 identity, bit 3 inline,
// bits 4-5 nbytes-1, 6-7 nchars-1, 8-31 the bytes; longer ones keep the pool
// offset in bits 8-31.  Canonical-ordering entries (file bit 4: kept marks with
// their ccc in bits 8-15, precomposed chars holding them, removed starters) are
// never inlined, so on the device (e & 24) == 16 identifies them.  Plus a flat
// copy of the BMP so one load resolves it.
static void to_device_entries(HostTokenizer &t) {
    for (uint32_t &e : t.uentry) {
        const uint32_t cls = e & 3u;
        // bit 4 (canonical ordering) entries stay as they are: (e & 24) == 16 marks them
        if ((e & 4u) || (e & 16u) || cls == UC_WS || cls == UC_DEL) continue;
        const uint32_t off = e >> 8;
        const uint32_t nb = t.upool[off], nc = t.upool[off + 1];
        if (nb >= 1 && nb <= 3 && nc >= 1 && nc <= 4) {
            uint32_t bytes = 0;
            for (uint32_t k = 0; k < nb; ++k) bytes |= (uint32_t)t.upool[off + 2 + k] << (8 * k);
            if (bytes >> 24) continue;
            e = cls | 8u | ((nb - 1) << 4) | ((nc - 1) << 6) | (bytes << 8);
        }
    }
    t.ubmp.assign(2 * 0x10000, 0u);  // (entry, WordPiece ISO id: wp_iso_ids) per code point
    for (uint32_t cp = 0; cp < 0x10000; ++cp) t.ubmp[2 * cp] = t.uentry[(size_t)t.upage[cp >> 7] * 128 + (cp & 127)];
}

// ---------------------------------------------------------------------------
// Byte-level BPE (gpt2): tokenizers' ByteLevel pre-tokenizer + BPE model.
// ---------------------------------------------------------------------------

// GPT-2 bytes_to_unicode(): byte -> code point of its printable stand-in
static std::vector<uint32_t> byte_to_cp() {
    std::vector<uint32_t> m(256, 0);
    std::vector<bool> direct(256, false);
    for (uint32_t b = '!'; b <= '~'; ++b) direct[b] = true;
    for (uint32_t b = 0xA1; b <= 0xAC; ++b) direct[b] = true;
    for (uint32_t b = 0xAE; b <= 0xFF; ++b) direct[b] = true;
    uint32_t n = 0;
    for (uint32_t b = 0; b < 256; ++b) m[b] = direct[b] ? b : 256 + n++;
    return m;
}

static void utf8_append(std::string &o, uint32_t cp) {
    if (cp < 0x80) o += (char)cp;
    else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 63)); }
    else if (cp < 0x10000) {
        o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 63)); o += (char)(0x80 | (cp & 63));
    } else {
        o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 63));
        o += (char)(0x80 | ((cp >> 6) & 63)); o += (char)(0x80 | (cp & 63));
    }
}

// The one-char WordPiece id of every BMP char k_wordpiece_chunks' rare pass would probe
// itself -- ISO class, not a canonical-ordering entry, normalizing to one char (identity:
// the char's own UTF-8; inline: the entry's bytes) -- as bit 31 | the id of that string as a
// non-"##" piece of <= maxlen_first bytes, else of [UNK]; 0 for every other char.  The rare
// pass reads it with the char's entry, so such a char costs one load and no probe.
static void wp_iso_ids(HostTokenizer &t) {
    std::unordered_map<std::string, int> ids;
    for (size_t i = 0; i < t.pieces.size(); ++i) ids[t.pieces[i]] = (int)i;  // (a duplicate keeps its last id)
    for (uint32_t cp = 0x80; cp < 0x10000; ++cp) {
        const uint32_t e = t.ubmp[2 * cp];
        if ((e & 3u) != UC_ISO || (e & 24u) == 16u || !((e & 4u) || ((e & 8u) && ((e >> 6) & 3u) == 0u))) continue;
        std::string w;
        if (e & 4u) utf8_append(w, cp);
        else
            for (uint32_t q = 0; q <= ((e >> 4) & 3u); ++q) w += (char)((e >> (8 + 8 * q)) & 0xFFu);
        int id = -1;
        if ((int)w.size() <= t.maxlen_first) {
            const auto it = ids.find(w);
            if (it != ids.end()) id = it->second;
        }
        t.ubmp[2 * cp + 1] = 0x80000000u | (uint32_t)(id >= 0 ? id : t.unk_id);
    }
}

// byte-level token string -> raw bytes (false if a char is not a byte stand-in)
static bool token_bytes(const std::string &tok, const std::unordered_map<uint32_t, uint8_t> &rev, std::string &out) {
    out.clear();
    size_t i = 0;
    while (i < tok.size()) {
        const uint8_t b = (uint8_t)tok[i];
        uint32_t cp;
        int n;
        if (b < 0x80) { cp = b; n = 1; }
        else if ((b & 0xE0) == 0xC0) { cp = b & 0x1F; n = 2; }
        else if ((b & 0xF0) == 0xE0) { cp = b & 0x0F; n = 3; }
        else { cp = b & 0x07; n = 4; }
        if (i + n > tok.size()) return false;
        for (int k = 1; k < n; ++k) cp = (cp << 6) | ((uint8_t)tok[i + k] & 0x3F);
        auto it = rev.find(cp);
        if (it == rev.end()) return false;
        out += (char)it->second;
        i += n;
    }
    return true;
}

static uint32_t merge_lookup(const HostTokenizer &t, uint32_t a, uint32_t b) {
    const uint32_t key = a << 16 | b, h = merge_hash(key);
    const MSlot &s1 = t.mslots[cuckoo_slot1(h, t.mslot_mask)];
    if (s1.key == key) return s1.val;
    const MSlot &s2 = t.mslots[cuckoo_slot2(h, t.mslot_mask)];
    if (s2.key == key) return s2.val;
    return 0xFFFFFFFFu;
}

// tokenizers' Word::merge_all: a min-heap of (rank, position) over live pairs,
// stale entries skipped (models/bpe/word.rs).
std::vector<int> bpe_encode_bytes(const HostTokenizer &t, const uint8_t *s, size_t n) {
    struct Sym { int id, prev, next; bool live; };
    std::vector<Sym> sym(n);
    for (size_t i = 0; i < n; ++i) sym[i] = {t.byte_id[s[i]], (int)i - 1, i + 1 < n ? (int)i + 1 : -1, true};
    typedef std::pair<uint64_t, uint32_t> Ent;  // (rank << 32 | pos, merged id)
    std::priority_queue<Ent, std::vector<Ent>, std::greater<Ent>> q;
    auto push = [&](int pos) {
        if (pos < 0 || sym[pos].next < 0) return;
        const uint32_t v = merge_lookup(t, (uint32_t)sym[pos].id, (uint32_t)sym[sym[pos].next].id);
        if (v != 0xFFFFFFFFu) q.push({(uint64_t)(v >> 16) << 32 | (uint32_t)pos, v & 0xFFFFu});
    };
    for (size_t i = 0; i + 1 < n; ++i) push((int)i);
    while (!q.empty()) {
        const Ent e = q.top();
        q.pop();
        const int pos = (int)(uint32_t)e.first;
        if (!sym[pos].live || sym[pos].next < 0) continue;
        const int nx = sym[pos].next;
        const uint32_t v = merge_lookup(t, (uint32_t)sym[pos].id, (uint32_t)sym[nx].id);
        if (v == 0xFFFFFFFFu || (v & 0xFFFFu) != e.second) continue;  // expired entry
        sym[pos].id = (int)e.second;
        sym[nx].live = false;
        sym[pos].next = sym[nx].next;
        if (sym[pos].next >= 0) sym[sym[pos].next].prev = pos;
        push(sym[pos].prev);
        push(pos);
    }
    std::vector<int> out;
    for (size_t i = 0; i < n; ++i)
        if (sym[i].live) out.push_back(sym[i].id);
    return out;
}

static void load_gpt2_classes(const std::string &path, HostTokenizer &t) {
    const std::string b = read_file(path);
    if (b.size() < 16 || b.compare(0, 4, "SDLG") != 0) throw std::runtime_error("bad class table " + path);
    uint32_t ver, np, nb;
    std::memcpy(&ver, &b[4], 4);
    std::memcpy(&np, &b[8], 4);
    std::memcpy(&nb, &b[12], 4);
    if (ver != 1 || np != 0x110000 / 256 || b.size() != 16 + 2 * (size_t)np + 64 * (size_t)nb)
        throw std::runtime_error("bad class table " + path);
    t.gpage.resize(np);
    std::memcpy(t.gpage.data(), &b[16], 2 * (size_t)np);
    t.gblock.assign(b.begin() + 16 + 2 * np, b.end());
    // the kernels classify ASCII arithmetically: check it is the table's
    for (uint32_t c = 0; c < 128; ++c) {
        const uint32_t k = (t.gblock[(size_t)t.gpage[0] * 64 + (c >> 2)] >> (2 * (c & 3))) & 3u;
        uint32_t want = GC_O;
        if ((c | 0x20u) - 'a' < 26u) want = GC_L;
        else if (c - '0' < 10u) want = GC_N;
        else if (c == ' ' || (c >= 9 && c <= 13)) want = GC_W;
        if (k != want) throw std::runtime_error("gpt2 class table: ASCII classes differ from the kernels' classifier");
    }
}

static void load_byte_bpe(const JValue &root, const std::string &data_dir, HostTokenizer &t) {
    const JValue *model = root.get("model");
    auto is_null_or = [](const JValue *v, const char *s) { return !v || v->kind == JValue::NUL || v->is_str(s); };
    auto is_true = [](const JValue *v) { return v && v->kind == JValue::BOOL && v->b; };
    if (model->get("dropout") && model->get("dropout")->kind == JValue::NUM)
        throw std::runtime_error("BPE dropout unsupported (non-deterministic)");
    if (!is_null_or(model->get("continuing_subword_prefix"), "") || !is_null_or(model->get("end_of_word_suffix"), ""))
        throw std::runtime_error("byte-level BPE with subword prefix/suffix unsupported");
    if (is_true(model->get("byte_fallback")) || is_true(model->get("ignore_merges")))
        throw std::runtime_error("BPE byte_fallback/ignore_merges unsupported");
    const JValue *norm = root.get("normalizer");
    if (norm && norm->kind != JValue::NUL) throw std::runtime_error("byte-level BPE: normalizer must be null (gpt2)");
    const JValue *pre = root.get("pre_tokenizer");
    if (!pre || !pre->get("type") || !pre->get("type")->is_str("ByteLevel") || is_true(pre->get("add_prefix_space")) ||
        (pre->get("use_regex") && !is_true(pre->get("use_regex"))))
        throw std::runtime_error("pre_tokenizer must be ByteLevel(add_prefix_space=false, use_regex=true)");
    const JValue *pp = root.get("post_processor");
    if (pp && pp->kind != JValue::NUL && !(pp->get("type") && pp->get("type")->is_str("ByteLevel")))
        throw std::runtime_error("post_processor must be ByteLevel or null (no ids added)");
    t.kind = TOK_BYTE_BPE;
    const JValue *vocab = model->get("vocab");
    if (!vocab || vocab->kind != JValue::OBJ) throw std::runtime_error("model.vocab missing");
    int max_id = -1;
    for (auto &kv : vocab->obj) max_id = std::max(max_id, (int)kv.second.num);
    t.pieces.assign((size_t)max_id + 1, std::string());
    std::unordered_map<std::string, int> id_of;
    for (auto &kv : vocab->obj) {
        t.pieces[(size_t)kv.second.num] = kv.first;
        id_of[kv.first] = (int)kv.second.num;
    }
    const JValue *added = root.get("added_tokens");
    if (added && added->kind == JValue::ARR) {
        for (auto &a : added->arr) {
            const JValue *c = a.get("content"), *id = a.get("id");
            if (!c || !id) continue;
            // no normalizer: a normalized added token matches the raw text too
            if (is_true(a.get("lstrip")) || is_true(a.get("rstrip")) || is_true(a.get("single_word")))
                throw std::runtime_error("added token options (lstrip/rstrip/single_word) unsupported");
            t.added.emplace_back(c->str, (int)id->num);
            if ((size_t)id->num >= t.pieces.size()) t.pieces.resize((size_t)id->num + 1);
            if (t.pieces[(size_t)id->num].empty()) t.pieces[(size_t)id->num] = c->str;
            id_of.emplace(c->str, (int)id->num);
        }
    }
    if (t.pieces.size() > 65535) throw std::runtime_error("vocabulary larger than 65535 ids is not supported");
    auto eos = id_of.find("<|endoftext|>");
    if (eos == id_of.end()) throw std::runtime_error("gpt2 tokenizer lacks <|endoftext|>");
    t.eos_id = eos->second;
    // byte symbols
    const std::vector<uint32_t> b2c = byte_to_cp();
    std::unordered_map<uint32_t, uint8_t> rev;
    t.byte_id.assign(256, 0);
    for (uint32_t b = 0; b < 256; ++b) {
        rev[b2c[b]] = (uint8_t)b;
        std::string u;
        utf8_append(u, b2c[b]);
        auto it = id_of.find(u);
        if (it == id_of.end()) throw std::runtime_error("byte-level vocab lacks a byte symbol");
        t.byte_id[b] = (uint16_t)it->second;
    }
    // merges: rank = position; (left, right) -> merged
    const JValue *merges = model->get("merges");
    if (!merges || merges->kind != JValue::ARR) throw std::runtime_error("model.merges missing");
    const size_t nm = merges->arr.size();
    if (nm >= MERGE_NONE) throw std::runtime_error("too many merges (rank must fit 16 bits)");
    std::vector<std::array<uint32_t, 3>> ms;
    ms.reserve(nm);
    std::vector<int64_t> max_creator(t.pieces.size(), -1);
    for (size_t r = 0; r < nm; ++r) {
        const JValue &m = merges->arr[r];
        std::string a, b;
        if (m.kind == JValue::STR) {
            const size_t sp = m.str.find(' ', 1);
            if (sp == std::string::npos) throw std::runtime_error("bad merge entry");
            a = m.str.substr(0, sp);
            b = m.str.substr(sp + 1);
        } else if (m.kind == JValue::ARR && m.arr.size() == 2) {
            a = m.arr[0].str;
            b = m.arr[1].str;
        } else {
            throw std::runtime_error("bad merge entry");
        }
        auto ia = id_of.find(a), ib = id_of.find(b), ic = id_of.find(a + b);
        if (ia == id_of.end() || ib == id_of.end() || ic == id_of.end())
            throw std::runtime_error("merge references a token missing from the vocab");
        ms.push_back({(uint32_t)ia->second, (uint32_t)ib->second, (uint32_t)ic->second});
        max_creator[(size_t)ic->second] = std::max<int64_t>(max_creator[(size_t)ic->second], (int64_t)r);
    }
    // The device merges every occurrence of the lowest-rank pair per step; that
    // equals tokenizers' heap order when a merge's parts are only created by
    // lower-ranked merges (true of any trained BPE).
    for (size_t r = 0; r < nm; ++r)
        if (max_creator[ms[r][0]] >= (int64_t)r || max_creator[ms[r][1]] >= (int64_t)r)
            throw std::runtime_error("merges are not rank-monotone (a part is created by a later merge)");
    uint32_t slots = 1;
    while (slots < 4 * std::max<size_t>(nm, 1)) slots <<= 1;
    for (;; slots <<= 1) {
        t.mslot_mask = slots - 1;
        t.mslots.assign(slots, MSlot{0xFFFFFFFFu, 0});
        bool ok = true;
        for (size_t r = 0; r < nm && ok; ++r) {
            MSlot v{ms[r][0] << 16 | ms[r][1], (uint32_t)r << 16 | ms[r][2]};
            if (merge_lookup(t, ms[r][0], ms[r][1]) != 0xFFFFFFFFu) continue;  // duplicate pair keeps the first rank
            uint32_t pos = cuckoo_slot1(merge_hash(v.key), t.mslot_mask);
            bool placed = false;
            for (int kick = 0; kick < 2000; ++kick) {
                if (t.mslots[pos].key == 0xFFFFFFFFu) { t.mslots[pos] = v; placed = true; break; }
                std::swap(v, t.mslots[pos]);
                const uint32_t h = merge_hash(v.key);
                const uint32_t a = cuckoo_slot1(h, t.mslot_mask), b = cuckoo_slot2(h, t.mslot_mask);
                pos = pos == a ? b : a;
            }
            ok = placed;
        }
        if (ok) break;
        if (slots >= (1u << 24)) throw std::runtime_error("merge table build failed");
    }
    // word table: vocab strings whose own BPE is exactly themselves
    std::vector<bool> is_added(t.pieces.size(), false);
    for (auto &a : t.added) is_added[(size_t)a.second] = true;
    std::vector<VSlot> entries;
    t.vpool.clear();
    t.maxlen_first = t.maxlen_cont = 0;
    std::string bytes;
    for (auto &kv : vocab->obj) {
        const int id = (int)kv.second.num;
        if (is_added[(size_t)id] || id_of[kv.first] != id || !token_bytes(kv.first, rev, bytes)) continue;
        if (bytes.empty() || bytes.size() > 255) continue;
        const std::vector<int> enc = bpe_encode_bytes(t, (const uint8_t *)bytes.data(), bytes.size());
        if (enc.size() != 1 || enc[0] != id) continue;
        t.maxlen_first = std::max(t.maxlen_first, (int)bytes.size());
        VSlot v{};
        v.key = (uint32_t)bytes.size();
        v.id = (int32_t)id;
        v.pool_off = (uint32_t)t.vpool.size();
        v.hash = piece_hash((const uint8_t *)bytes.data(), bytes.size(), 0u);
        std::memcpy(v.inl, bytes.data(), std::min<size_t>(16, bytes.size()));
        t.vpool.insert(t.vpool.end(), bytes.begin(), bytes.end());
        entries.push_back(v);
    }
    t.word_table_entries = entries.size();
    t.vpool.resize(t.vpool.size() + 64, 0);
    slots = 1;
    while (slots < 4 * entries.size()) slots <<= 1;
    for (;; slots <<= 1) {
        t.slot_mask = slots - 1;
        t.slots.assign(slots, VSlot{0, -1, 0, 0, {0}});
        bool ok = true;
        for (const VSlot &v : entries)
            if (!cuckoo_insert(t.slots, t.slot_mask, v)) { ok = false; break; }
        if (ok) break;
        if (slots >= (1u << 24)) throw std::runtime_error("cuckoo table build failed");
    }
    set_added(t);
    if (t.opener && (t.opener >= 0x80 || (t.opener | 0x20u) - 'a' < 26u || t.opener - '0' < 10u))
        throw std::runtime_error("added tokens must start with an ASCII non-alphanumeric byte");
    for (auto &a : t.added)
        for (unsigned char ch : a.first)
            if (ch >= 0x80) throw std::runtime_error("byte-level BPE: added tokens must be ASCII");
    load_gpt2_classes(data_dir + "/gpt2_classes.bin", t);
}

// ---------------------------------------------------------------------------
// Unigram (t5-small): Precompiled normalizer + WhitespaceSplit + Metaspace +
// Unigram model + "$A </s>" (hub tokenizer.json layout).
// ---------------------------------------------------------------------------
static std::vector<uint8_t> b64decode(const std::string &s) {
    std::vector<uint8_t> o;
    uint32_t acc = 0;
    int bits = 0;
    for (unsigned char c : s) {
        int v = c >= 'A' && c <= 'Z' ? c - 'A' : c >= 'a' && c <= 'z' ? c - 'a' + 26 : c >= '0' && c <= '9' ? c - '0' + 52
              : c == '+' ? 62 : c == '/' ? 63 : -1;
        if (v < 0) continue;
        acc = acc << 6 | (uint32_t)v;
        bits += 6;
        if (bits >= 8) {
            bits -= 8;
            o.push_back((uint8_t)(acc >> bits));
        }
    }
    return o;
}

static VSlot make_slot(const std::string &pay, uint32_t cont, int32_t id, std::vector<uint8_t> &pool) {
    VSlot v{};
    v.key = (uint32_t)pay.size() | (cont << 8);
    v.id = id;
    v.pool_off = (uint32_t)pool.size();
    v.hash = piece_hash((const uint8_t *)pay.data(), pay.size(), cont);
    std::memcpy(v.inl, pay.data(), std::min<size_t>(16, pay.size()));
    pool.insert(pool.end(), pay.begin(), pay.end());
    return v;
}

// load <= 0.5 (two choices, one slot per bucket); the Unigram pieces table
// (probed by every Viterbi candidate) is kept apart from the word table so it
// stays small enough to live in L2
static void build_cuckoo(std::vector<VSlot> &tab, uint32_t &mask, const std::vector<VSlot> &entries) {
    uint32_t slots = 1;
    while (slots < 2 * entries.size()) slots <<= 1;
    for (;; slots <<= 1) {
        mask = slots - 1;
        tab.assign(slots, VSlot{0, -1, 0, 0, {0}});
        bool ok = true;
        for (const VSlot &v : entries)
            if (!cuckoo_insert(tab, mask, v)) { ok = false; break; }
        if (ok) break;
        if (slots >= (1u << 24)) throw std::runtime_error("cuckoo table build failed");
    }
}

// host probe of the vocab table (same slots the kernels read)
static int host_probe(const HostTokenizer &t, const uint8_t *pay, size_t n, uint32_t cont) {
    const uint32_t h = piece_hash(pay, n, cont);
    const uint32_t key = (uint32_t)n | (cont << 8);
    for (uint32_t s : {cuckoo_slot1(h, t.slot_mask), cuckoo_slot2(h, t.slot_mask)}) {
        const VSlot &v = t.slots[s];
        if (v.id >= 0 && v.key == key && std::memcmp(&t.vpool[v.pool_off], pay, n) == 0) return v.id;
    }
    return -1;
}

static const uint8_t kMeta[3] = {0xE2, 0x96, 0x81};  // U+2581

std::vector<int> unigram_encode_word(const HostTokenizer &t, const uint8_t *w, size_t n) {
    std::vector<uint8_t> b(kMeta, kMeta + 3);
    b.insert(b.end(), w, w + n);
    auto acc = [&](int i) -> uint32_t { return b[(size_t)i]; };
    auto cand = [&](int s, int e, double *sc) -> int {
        int id;
        if (s == 0) id = e >= 3 ? host_probe(t, b.data() + 3, (size_t)(e - 3), UC_META) : -1;
        else id = host_probe(t, b.data() + s, (size_t)(e - s), UC_PIECE);
        if (id >= 0) *sc = t.uscore[(size_t)id];
        return id;
    };
    struct Nodes {
        std::vector<UniNode> v;
        void set(int i, double s, int st, int id) { v[(size_t)i] = UniNode{s, st, id}; }
        double score(int i) const { return v[(size_t)i].score; }
        int start(int i) const { return v[(size_t)i].start; }
        int id(int i) const { return v[(size_t)i].id; }
    } nodes{std::vector<UniNode>(b.size() + 1)};
    std::vector<int> out;
    const int k = unigram_viterbi(acc, (int)b.size(), cand, nodes, t.unk_score, t.unk_id, t.maxlen_piece,
                                  [&](int i, int id) {
                                      if ((int)out.size() <= i) out.resize((size_t)i + 1);
                                      out[(size_t)i] = id;
                                  });
    out.resize((size_t)k);
    return out;
}

static void load_t5_props(const std::string &path, HostTokenizer &t) {
    const std::string b = read_file(path);
    if (b.size() < 16 || b.compare(0, 4, "SDLU") != 0) throw std::runtime_error("bad grapheme table " + path);
    uint32_t ver, np, nb;
    std::memcpy(&ver, &b[4], 4);
    std::memcpy(&np, &b[8], 4);
    std::memcpy(&nb, &b[12], 4);
    if (ver != 1 || np != 0x110000 / 256 || b.size() != 16 + 2 * (size_t)np + 256 * (size_t)nb)
        throw std::runtime_error("bad grapheme table " + path);
    t.tpage.resize(np);
    std::memcpy(t.tpage.data(), &b[16], 2 * (size_t)np);
    t.tblock.assign(b.begin() + 16 + 2 * np, b.end());
}

static void load_unigram(const JValue &root, const std::string &data_dir, HostTokenizer &t) {
    auto is_true = [](const JValue *v) { return v && v->kind == JValue::BOOL && v->b; };
    const JValue *model = root.get("model");
    if (is_true(model->get("byte_fallback"))) throw std::runtime_error("Unigram byte_fallback unsupported");
    // normalizer: Precompiled (the hub t5 layout)
    const JValue *norm = root.get("normalizer");
    if (!norm || !norm->get("type") || !norm->get("type")->is_str("Precompiled") || !norm->get("precompiled_charsmap"))
        throw std::runtime_error("Unigram: normalizer must be Precompiled (t5-small layout)");
    // pre_tokenizer: Sequence[WhitespaceSplit, Metaspace("▁", prefix)]
    const JValue *pre = root.get("pre_tokenizer");
    const JValue *seq = pre ? pre->get("pretokenizers") : nullptr;
    bool pre_ok = pre && pre->get("type") && pre->get("type")->is_str("Sequence") && seq && seq->kind == JValue::ARR &&
                  seq->arr.size() == 2 && seq->arr[0].get("type") && seq->arr[0].get("type")->is_str("WhitespaceSplit") &&
                  seq->arr[1].get("type") && seq->arr[1].get("type")->is_str("Metaspace");
    if (pre_ok) {
        const JValue &ms = seq->arr[1];
        const JValue *rep = ms.get("replacement"), *aps = ms.get("add_prefix_space"), *ps = ms.get("prepend_scheme");
        const JValue *split = ms.get("split");
        pre_ok = rep && rep->is_str("\xe2\x96\x81") && (is_true(aps) || (ps && ps->is_str("always"))) &&
                 (!split || is_true(split));
    }
    if (!pre_ok)
        throw std::runtime_error("Unigram: pre_tokenizer must be Sequence[WhitespaceSplit, Metaspace(U+2581, prefix)]");
    const JValue *vocab = model->get("vocab"), *unk = model->get("unk_id");
    if (!vocab || vocab->kind != JValue::ARR || !unk || unk->kind != JValue::NUM)
        throw std::runtime_error("Unigram: model.vocab / unk_id missing");
    t.kind = TOK_UNIGRAM;
    const size_t nv = vocab->arr.size();
    if (nv > 65535) throw std::runtime_error("vocabulary larger than 65535 ids is not supported");
    t.pieces.resize(nv);
    t.uscore.resize(nv);
    double min_score = INFINITY;
    for (size_t i = 0; i < nv; ++i) {
        const JValue &e = vocab->arr[i];
        if (e.kind != JValue::ARR || e.arr.size() != 2 || e.arr[0].kind != JValue::STR || e.arr[1].kind != JValue::NUM)
            throw std::runtime_error("Unigram: bad vocab entry");
        t.pieces[i] = e.arr[0].str;
        t.uscore[i] = e.arr[1].num;
        min_score = std::min(min_score, t.uscore[i]);
        t.maxlen_piece = std::max(t.maxlen_piece, (int)t.pieces[i].size());
    }
    t.unk_id = (int)unk->num;
    if (t.unk_id < 0 || (size_t)t.unk_id >= nv) throw std::runtime_error("Unigram: unk_id out of range");
    // The kernels keep a candidate's score as the nearest f32; a piece whose f64 is one ulp
    // off it is marked by bit 15 of its id in the device slot, the direction by the sign of
    // the stored f32 (sdl_batcher.cpp, tokenize_unigram.hip uni_score64), which restores the
    // exact f64. So such a piece needs an id < 32768 (t5-small: 32,100 pieces); a vocabulary
    // with a marked piece above that is refused at create (INTEGRATION.md "Limits").
    // Scores written from sentencepiece's f32 (hub tokenizer.json: 17-digit
    // decimals) come back from serde_json's two-rounding parse (json.hpp) as
    // that f32 or one f64 ulp away from it; anything further is refused.
    t.uscore32.resize(nv);
    t.uscore_adj.resize(nv);
    for (size_t i = 0; i < nv; ++i) {
        const float f = (float)t.uscore[i];
        int64_t bd, bf;
        const double df = (double)f;
        std::memcpy(&bd, &t.uscore[i], 8);
        std::memcpy(&bf, &df, 8);
        const int64_t adj = bd - bf;
        if (adj < -1 || adj > 1 || std::isnan(t.uscore[i]))
            throw std::runtime_error("Unigram: piece scores must be within one f64 ulp of an f32 value");
        t.uscore32[i] = f;
        t.uscore_adj[i] = (int8_t)adj;
    }
    t.unk_score = min_score - 10.0;  // K_UNK_PENALTY
    // added tokens: "<...>" with no other '<' / '>' inside (so a match ends at the first '>')
    std::unordered_map<std::string, int> id_of;
    for (size_t i = 0; i < nv; ++i) id_of[t.pieces[i]] = (int)i;  // HashMap: a duplicate keeps the last id
    const JValue *added = root.get("added_tokens");
    if (added && added->kind == JValue::ARR) {
        for (auto &a : added->arr) {
            const JValue *c = a.get("content"), *id = a.get("id");
            if (!c || !id) continue;
            if (is_true(a.get("lstrip")) || is_true(a.get("rstrip")) || is_true(a.get("single_word")) ||
                is_true(a.get("normalized")))
                throw std::runtime_error("added token options (normalized/lstrip/rstrip/single_word) unsupported");
            const std::string &s = c->str;
            if (s.size() < 2 || (int)s.size() > MAX_SPECIAL_LEN || s.front() != '<' || s.back() != '>' ||
                s.find('<', 1) != std::string::npos || s.find('>') != s.size() - 1)
                throw std::runtime_error("Unigram: added tokens must look like <...>");
            t.added.emplace_back(s, (int)id->num);
        }
    }
    // post_processor "$A </s>"
    const JValue *pp = root.get("post_processor");
    const JValue *single = pp ? pp->get("single") : nullptr;
    if (!pp || !pp->get("type") || !pp->get("type")->is_str("TemplateProcessing") || !single ||
        single->kind != JValue::ARR || single->arr.size() != 2 || !single->arr[0].get("Sequence") ||
        !single->arr[1].get("SpecialToken"))
        throw std::runtime_error("Unigram: post_processor must be TemplateProcessing \"$A </s>\"");
    {
        const std::string eos = single->arr[1].get("SpecialToken")->get("id")->str;
        const JValue *spt = pp->get("special_tokens");
        const JValue *ent = spt ? spt->get(eos) : nullptr;
        const JValue *ids = ent ? ent->get("ids") : nullptr;
        if (!ids || ids->kind != JValue::ARR || ids->arr.size() != 1)
            throw std::runtime_error("Unigram: template special token must have one id");
        t.tpl_eos = (int)ids->arr[0].num;
    }
    auto find_added = [&](const std::string &s) {
        for (auto &a : t.added)
            if (a.first == s) return a.second;
        auto it = id_of.find(s);
        return it == id_of.end() ? -1 : it->second;
    };
    t.eos_id = find_added("</s>");  // TokenizerInfo.eos (tokenizer_wrapper.rs:81-88)
    t.pad_id = find_added("<pad>");
    if (t.eos_id < 0) throw std::runtime_error("t5 tokenizer lacks </s>");
    t.extra_ids.resize(100);
    for (int k = 0; k < 100; ++k) {
        t.extra_ids[(size_t)k] = find_added("<extra_id_" + std::to_string(k) + ">");
        if (t.extra_ids[(size_t)k] < 0) throw std::runtime_error("t5 tokenizer lacks <extra_id_" + std::to_string(k) + ">");
    }
    // charsmap
    const std::vector<uint8_t> cm = b64decode(norm->get("precompiled_charsmap")->str);
    uint32_t tsize = 0;
    if (cm.size() < 4) throw std::runtime_error("bad precompiled_charsmap");
    std::memcpy(&tsize, cm.data(), 4);
    if (tsize % 4 || 4 + (size_t)tsize > cm.size()) throw std::runtime_error("bad precompiled_charsmap");
    t.trie.resize(tsize / 4);
    std::memcpy(t.trie.data(), cm.data() + 4, tsize);
    t.tnorm.assign(cm.begin() + 4 + tsize, cm.end());
    t.tnorm.push_back(0);
    load_t5_props(data_dir + "/t5_graphemes.bin", t);
    // What the kernels assume of the charsmap (checked, else refused):
    //  - printable ASCII bytes are not changed (a simple ASCII word is its own
    //    normalization: each of its clusters is one ASCII char);
    //  - \t \n \f \r map to non-empty whitespace and ' ' to itself (they separate words);
    //  - no key starts with ' ' or with a Prepend char (a cluster across a word
    //    edge then falls back to per-char lookups, so words normalize apart).
    auto lookup = [&](const uint8_t *s, int n) {
        return trie_shortest(t.trie.data(), (uint32_t)t.trie.size(), [&](int i) -> uint32_t { return s[i]; }, n);
    };
    auto norm_at = [&](int32_t off) { return std::string((const char *)&t.tnorm[(size_t)off]); };
    for (uint32_t b = 0x21; b < 0x7F; ++b) {
        const uint8_t c = (uint8_t)b;
        const int32_t r = lookup(&c, 1);
        if (r >= 0 && norm_at(r) != std::string(1, (char)b))
            throw std::runtime_error("charsmap changes printable ASCII (unsupported by the kernels)");
    }
    for (uint8_t c : {(uint8_t)9, (uint8_t)10, (uint8_t)12, (uint8_t)13, (uint8_t)32}) {
        const int32_t r = lookup(&c, 1);
        std::string m = r >= 0 ? norm_at(r) : std::string(1, (char)c);
        bool ws = !m.empty();
        for (unsigned char x : m) ws = ws && (x == ' ' || (x >= 9 && x <= 13));
        if (!ws) throw std::runtime_error("charsmap must keep ASCII whitespace whitespace");
    }
    {
        // first bytes of every key: walk the root's children
        const uint32_t root_pos = du_offset(t.trie[0]);
        for (uint32_t c = 1; c < 256; ++c) {
            const uint32_t p = root_pos ^ c;
            if (p >= t.trie.size() || (t.trie[p] & ((1u << 31) | 0xFFu)) != c) continue;
            if (c == 0x20) throw std::runtime_error("charsmap has a key starting with ' '");
        }
        // keys starting with a Prepend char: probe every Prepend code point's bytes as a key prefix
        for (uint32_t cp = 0x80; cp < 0x110000; ++cp) {
            if ((cp >= 0xD800 && cp < 0xE000) || (gprop(t.tpage.data(), t.tblock.data(), cp) & 15u) != GB_PREPEND) continue;
            std::string u;
            utf8_append(u, cp);
            uint32_t pos = root_pos;
            bool path = true;
            for (unsigned char c : u) {
                pos ^= c;
                if (pos >= t.trie.size() || (t.trie[pos] & ((1u << 31) | 0xFFu)) != c) { path = false; break; }
                pos ^= du_offset(t.trie[pos]);
            }
            if (path) throw std::runtime_error("charsmap has a key starting with a Prepend char");
        }
    }
    // per-code-point normalizer entries (the device resolves a one-char cluster
    // with one load; only multi-char clusters starting with a key prefix walk the trie)
    {
        const uint32_t root_pos = du_offset(t.trie[0]);
        t.cpage.assign(0x110000 / 256, 0);
        t.cent.clear();
        std::unordered_map<std::string, uint16_t> seen;
        std::vector<uint32_t> blk(512);
        for (uint32_t pg = 0; pg < 0x110000 / 256; ++pg) {
            for (uint32_t lo = 0; lo < 256; ++lo) {
                const uint32_t cp = pg * 256 + lo;
                uint32_t x = gprop(t.tpage.data(), t.tblock.data(), cp), y = 0;
                if (!(cp >= 0xD800 && cp < 0xE000) && cp != 0) {
                    std::string u;
                    utf8_append(u, cp);
                    uint32_t pos = root_pos;
                    bool path = true;
                    int32_t val = -1;
                    for (size_t i = 0; i < u.size(); ++i) {
                        const uint32_t c = (uint8_t)u[i];
                        pos ^= c;
                        if (pos >= t.trie.size() || (t.trie[pos] & ((1u << 31) | 0xFFu)) != c) { path = false; break; }
                        const uint32_t unit = t.trie[pos];
                        pos ^= du_offset(unit);
                        if ((unit >> 8) & 1u) {
                            if (i + 1 == u.size()) val = (int32_t)(t.trie[pos] & 0x7FFFFFFFu);
                            else { path = false; break; }  // a key ending inside the char: never a prefix of text
                        }
                    }
                    if (path) {
                        if (val >= 0) {
                            x |= CP_KEY;
                            const char *ns = (const char *)&t.tnorm[(size_t)val];
                            const size_t nl = std::strlen(ns);
                            if (nl <= 4) {
                                x |= CP_INLINE | ((uint32_t)nl << 11);
                                for (size_t k = 0; k < nl; ++k) y |= (uint32_t)(uint8_t)ns[k] << (8 * k);
                            } else {
                                y = (uint32_t)val;
                            }
                        }
                        for (uint32_t c = 1; c < 256; ++c) {
                            const uint32_t q = pos ^ c;
                            if (q < t.trie.size() && (t.trie[q] & ((1u << 31) | 0xFFu)) == c) { x |= CP_PREFIX; break; }
                        }
                    }
                }
                blk[2 * lo] = x;
                blk[2 * lo + 1] = y;
            }
            const std::string key((const char *)blk.data(), blk.size() * 4);
            auto it = seen.find(key);
            if (it == seen.end()) {
                const size_t idx = t.cent.size() / 512;
                if (idx > 65535) throw std::runtime_error("code point table too large");
                it = seen.emplace(key, (uint16_t)idx).first;
                t.cent.insert(t.cent.end(), blk.begin(), blk.end());
            }
            t.cpage[pg] = it->second;
        }
    }
    // vocab table: pieces (UC_META "▁"+payload / UC_PIECE), added tokens, word table
    std::vector<VSlot> entries;
    t.vpool.clear();
    t.maxlen_first = t.maxlen_cont = 0;
    const std::string meta((const char *)kMeta, 3);
    for (size_t i = 0; i < nv; ++i) {
        const std::string &s = t.pieces[i];
        if (s.empty() || id_of[s] != (int)i) continue;
        const bool m = s.compare(0, 3, meta) == 0;
        const std::string pay = m ? s.substr(3) : s;
        if (pay.size() > 255) throw std::runtime_error("vocabulary piece longer than 255 bytes");
        if (m) t.maxlen_cont = std::max(t.maxlen_cont, (int)pay.size());
        else t.maxlen_first = std::max(t.maxlen_first, (int)pay.size());
        entries.push_back(make_slot(pay, m ? UC_META : UC_PIECE, (int32_t)i, t.vpool));
    }
    // the longest plain piece (>= 4 bytes) under each hashed 4-byte prefix: k_unigram_viterbi
    // skips a payload row's candidates of >= 4 bytes past it (a key collision only raises it)
    t.upfx.assign((size_t)1 << UNI_PFX_BITS, 0);
    for (size_t i = 0; i < nv; ++i) {
        const std::string &s = t.pieces[i];
        if (s.size() < 4 || id_of[s] != (int)i || s.compare(0, 3, meta) == 0) continue;
        uint32_t x;
        std::memcpy(&x, s.data(), 4);
        uint8_t &b = t.upfx[uni_pfx_key(x)];
        b = (uint8_t)std::max<size_t>(b, std::min<size_t>(s.size(), 255));
    }
    // candidate rows are 64-bit masks in the kernels
    if (t.maxlen_cont > 63 || t.maxlen_first > 64)
        throw std::runtime_error("Unigram: pieces longer than 64 bytes are not supported");
    for (auto &a : t.added) entries.push_back(make_slot(a.first, UC_ADDED, a.second, t.vpool));
    t.max_special_len = 0;
    for (auto &a : t.added) t.max_special_len = std::max(t.max_special_len, (int)a.first.size());
    t.opener = t.added.empty() ? 0u : (uint32_t)'<';
    build_cuckoo(t.slots, t.slot_mask, entries);  // pieces first: the word table's Viterbi probes them
    // word table: printable-ASCII words w -> Viterbi("▁w") ids, for w = every
    // "▁w" vocab piece and, up to UNI_WMAX bytes, w + "," and w + "." (a word
    // is its own normalization, so any entry is exact; comma/period-ended
    // words are the commonest word-table misses in running text)
    t.wres.clear();
    int maxw = 0;
    std::unordered_set<std::string> in_table;
    std::vector<VSlot> wentries;
    auto add_word = [&](const std::string &w) {
        if (!in_table.insert(w).second) return;
        const std::vector<int> ids = unigram_encode_word(t, (const uint8_t *)w.data(), w.size());
        if (ids.empty() || ids.size() > 127) return;
        int32_t packed;
        if (ids.size() == 1) {
            packed = (int32_t)((1u << 24) | (uint32_t)ids[0]);
        } else {
            packed = (int32_t)(((uint32_t)ids.size() << 24) | (uint32_t)t.wres.size());
            for (int x : ids) t.wres.push_back((uint16_t)x);
        }
        wentries.push_back(make_slot(w, UC_WORD, packed, t.vpool));
        maxw = std::max(maxw, (int)w.size());
    };
    std::vector<std::string> base_words;
    for (size_t i = 0; i < nv; ++i) {
        const std::string &s = t.pieces[i];
        if (s.size() <= 3 || s.compare(0, 3, meta) != 0 || id_of[s] != (int)i) continue;
        const std::string w = s.substr(3);
        bool ascii = w.size() <= 255;
        for (unsigned char c : w) ascii = ascii && c >= 0x21 && c <= 0x7E;
        if (!ascii) continue;
        add_word(w);
        if ((int)w.size() < UNI_WMAX) base_words.push_back(w);
    }
    for (const std::string &w : base_words) {
        add_word(w + ",");
        add_word(w + ".");
        // the next commonest word-table misses in running text: quoted,
        // parenthesised and colon/question/exclamation-ended words, possessives
        if ((int)w.size() + 2 <= UNI_WMAX) {
            for (const char *suf : {":", ";", "?", "!", ")", "\"", "'s", "),", ").", ".\"", ",\""})
                if ((int)(w.size() + std::strlen(suf)) <= UNI_WMAX) add_word(w + suf);
            add_word("\"" + w);
            add_word("(" + w);
        }
    }
    // sentence-initial and all-caps spellings of the base words (bare, and
    // comma/period-ended): a fifth of the held-out corpus's word-table misses,
    // and 50k entries that still fit the 2^20-slot table
    for (const std::string &w : base_words) {
        std::string cap = w, up = w;
        cap[0] = (char)std::toupper((unsigned char)cap[0]);
        for (char &c : up) c = (char)std::toupper((unsigned char)c);
        for (const std::string &v : {cap, up}) {
            if (v == w) continue;
            add_word(v);
            add_word(v + ",");
            add_word(v + ".");
        }
    }
    if (t.wres.size() >= (1u << 24)) throw std::runtime_error("word table too large");
    t.wres.push_back(0);
    t.word_table_entries = entries.size() + wentries.size();
    t.vpool.resize(t.vpool.size() + 64, 0);
    build_cuckoo(t.wslots, t.wslot_mask, wentries);
    t.max_word = maxw;
    // device slots: word 3 (the host's cuckoo hash) carries a piece's f32 score
    for (VSlot &v : t.slots) {
        const uint32_t cont = v.key >> 8;
        if (v.id >= 0 && (cont == UC_PIECE || cont == UC_META)) {
            float f = t.uscore32[(size_t)v.id];
            std::memcpy(&v.hash, &f, 4);
        }
    }
    // the kernels emit printable ASCII without a table load: it must be GCB Other
    for (uint32_t c = 0x21; c < 0x7F; ++c)
        if (gprop(t.tpage.data(), t.tblock.data(), c) != 0) throw std::runtime_error("unexpected ASCII grapheme class");
}

void load_tokenizer(const std::string &path, const std::string &data_dir, HostTokenizer &t) {
    const std::string body = read_file(path);
    const bool is_json = path.size() >= 5 && path.compare(path.size() - 5, 5, ".json") == 0;
    if (is_json) {
        JValue root = JParser(body).parse();
        const JValue *model = root.get("model");
        if (model && model->get("type") && model->get("type")->is_str("BPE")) {
            load_byte_bpe(root, data_dir, t);
            return;
        }
        if (model && model->get("type") && model->get("type")->is_str("Unigram")) {
            load_unigram(root, data_dir, t);
            return;
        }
        if (!model || !model->get("type") || !model->get("type")->is_str("WordPiece"))
            throw std::runtime_error("only WordPiece and byte-level BPE tokenizer.json models are supported");
        const JValue *pfx = model->get("continuing_subword_prefix");
        if (pfx && !pfx->is_str("##")) throw std::runtime_error("continuing_subword_prefix must be ##");
        const JValue *mx = model->get("max_input_chars_per_word");
        if (mx && mx->kind == JValue::NUM && (int)mx->num != MAX_WORD_CHARS)
            throw std::runtime_error("max_input_chars_per_word must be 100");
        if (!is_bert_normalizer(root.get("normalizer")))
            throw std::runtime_error("normalizer must be BertNormalizer(lowercase, strip accents, clean_text, chinese)");
        const JValue *pre = root.get("pre_tokenizer");
        if (!pre || !pre->get("type") || !pre->get("type")->is_str("BertPreTokenizer"))
            throw std::runtime_error("pre_tokenizer must be BertPreTokenizer");
        const JValue *vocab = model->get("vocab");
        if (!vocab || vocab->kind != JValue::OBJ) throw std::runtime_error("model.vocab missing");
        int max_id = -1;
        for (auto &kv : vocab->obj) max_id = std::max(max_id, (int)kv.second.num);
        t.pieces.assign((size_t)max_id + 1, std::string());
        for (auto &kv : vocab->obj) t.pieces[(size_t)kv.second.num] = kv.first;
        const JValue *unk = model->get("unk_token");
        std::string unk_s = unk && unk->kind == JValue::STR ? unk->str : "[UNK]";
        const JValue *added = root.get("added_tokens");
        if (added && added->kind == JValue::ARR) {
            for (auto &a : added->arr) {
                const JValue *c = a.get("content"), *id = a.get("id");
                auto b = [&](const char *k) { const JValue *v = a.get(k); return v && v->kind == JValue::BOOL && v->b; };
                if (!c || !id) continue;
                if (b("normalized") || b("lstrip") || b("rstrip") || b("single_word"))
                    throw std::runtime_error("added token options (normalized/lstrip/rstrip/single_word) unsupported");
                t.added.emplace_back(c->str, (int)id->num);
                if ((size_t)id->num >= t.pieces.size()) t.pieces.resize((size_t)id->num + 1);
                if (t.pieces[(size_t)id->num].empty()) t.pieces[(size_t)id->num] = c->str;
            }
        }
        // post-processor: [CLS] $A [SEP] (TemplateProcessing or BertProcessing)
        const JValue *pp = root.get("post_processor");
        auto id_of = [&](const std::string &s) {
            for (size_t i = 0; i < t.pieces.size(); ++i)
                if (t.pieces[i] == s) return (int)i;
            return -1;
        };
        t.unk_id = id_of(unk_s);
        if (pp && pp->get("type") && pp->get("type")->is_str("BertProcessing")) {
            t.tpl_cls = (int)pp->get("cls")->arr[1].num;
            t.tpl_sep = (int)pp->get("sep")->arr[1].num;
        } else if (pp && pp->get("type") && pp->get("type")->is_str("TemplateProcessing")) {
            const JValue *single = pp->get("single");
            if (!single || single->kind != JValue::ARR || single->arr.size() != 3)
                throw std::runtime_error("TemplateProcessing must be [CLS] $A [SEP]");
            const JValue *a0 = single->arr[0].get("SpecialToken"), *a2 = single->arr[2].get("SpecialToken");
            if (!a0 || !a2 || !single->arr[1].get("Sequence"))
                throw std::runtime_error("TemplateProcessing must be [CLS] $A [SEP]");
            t.tpl_cls = id_of(a0->get("id")->str);
            t.tpl_sep = id_of(a2->get("id")->str);
        } else {
            throw std::runtime_error("post_processor must add [CLS] ... [SEP]");
        }
    } else {
        // vocab.txt: one piece per line, id = line; BertWordPieceTokenizer defaults
        size_t s = 0;
        while (s < body.size()) {
            size_t e = body.find('\n', s);
            if (e == std::string::npos) e = body.size();
            size_t l = e - s;
            if (l && body[s + l - 1] == '\r') --l;
            t.pieces.push_back(body.substr(s, l));
            s = e + 1;
        }
        auto id_of = [&](const std::string &x) {
            for (size_t i = 0; i < t.pieces.size(); ++i)
                if (t.pieces[i] == x) return (int)i;
            return -1;
        };
        for (const char *sp : {"[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"}) {
            int id = id_of(sp);
            if (id >= 0) t.added.emplace_back(sp, id);
        }
        t.unk_id = id_of("[UNK]");
        t.tpl_cls = id_of("[CLS]");
        t.tpl_sep = id_of("[SEP]");
    }
    auto find = [&](const char *x) {
        for (size_t i = 0; i < t.pieces.size(); ++i)
            if (t.pieces[i] == x) return (int)i;
        return -1;
    };
    t.cls_id = find("[CLS]");
    t.sep_id = find("[SEP]");
    t.pad_id = find("[PAD]");
    t.mask_id = find("[MASK]");
    if (t.unk_id < 0 || t.cls_id < 0 || t.sep_id < 0 || t.tpl_cls < 0 || t.tpl_sep < 0)
        throw std::runtime_error("tokenizer lacks [UNK]/[CLS]/[SEP]");
    set_added(t);
    build_vocab_table(t);
    load_unicode(data_dir + "/bert_uncased_unicode.bin", t);
    check_ascii_and_ids(t);
    to_device_entries(t);
    wp_iso_ids(t);
}

}  // namespace sdl
