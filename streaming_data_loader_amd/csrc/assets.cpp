// assets.cpp -- loads the tokenizer the Batcher runs (tokenizer_holder.rs:64-97
// gets it from the HF hub with Tokenizer::from_pretrained; here the same
// tokenizer.json format is read from disk) and packs it for the device.
#include "assets.hpp"

#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <unordered_map>

#include "json.hpp"

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
    if (hdr[0] != 1) throw std::runtime_error("unicode table version mismatch");
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
    for (size_t id = 0; id < n; ++id) {
        const std::string &s = t.pieces[id];
        if (s.empty() || last[s] != (int)id) continue;
        const uint32_t cont = (s.size() > 2 && s[0] == '#' && s[1] == '#') ? 1u : 0u;
        const std::string pay = cont ? s.substr(2) : s;
        if (pay.size() > 255) throw std::runtime_error("vocabulary piece longer than 255 bytes");
        if (cont) t.maxlen_cont = std::max(t.maxlen_cont, (int)pay.size());
        else t.maxlen_first = std::max(t.maxlen_first, (int)pay.size());
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
// offset in bits 8-31.  Plus a flat copy of the BMP so one load resolves it.
static void to_device_entries(HostTokenizer &t) {
    for (uint32_t &e : t.uentry) {
        const uint32_t cls = e & 3u;
        if ((e & 4u) || cls == UC_WS || cls == UC_DEL) continue;
        const uint32_t off = e >> 8;
        const uint32_t nb = t.upool[off], nc = t.upool[off + 1];
        if (nb >= 1 && nb <= 3 && nc >= 1 && nc <= 4) {
            uint32_t bytes = 0;
            for (uint32_t k = 0; k < nb; ++k) bytes |= (uint32_t)t.upool[off + 2 + k] << (8 * k);
            if (bytes >> 24) continue;
            e = cls | 8u | ((nb - 1) << 4) | ((nc - 1) << 6) | (bytes << 8);
        }
    }
    t.ubmp.resize(0x10000);
    for (uint32_t cp = 0; cp < 0x10000; ++cp) t.ubmp[cp] = t.uentry[(size_t)t.upage[cp >> 7] * 128 + (cp & 127)];
}

void load_tokenizer(const std::string &path, const std::string &data_dir, HostTokenizer &t) {
    const std::string body = read_file(path);
    const bool is_json = path.size() >= 5 && path.compare(path.size() - 5, 5, ".json") == 0;
    if (is_json) {
        JValue root = JParser(body).parse();
        const JValue *model = root.get("model");
        if (!model || !model->get("type") || !model->get("type")->is_str("WordPiece"))
            throw std::runtime_error("only WordPiece tokenizer.json models are supported by this build");
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
}

}  // namespace sdl
