// assets.hpp -- tokenizer assets on the host, packed for the device.
#pragma once

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "common.hpp"

namespace sdl {

struct HostTokenizer {
    int kind = TOK_WORDPIECE;  // TOK_*
    // ---- what get_tokenizer(cfg) yields (tokenizer_wrapper.rs:162-189) -----
    std::vector<std::string> pieces;                   // id -> piece
    std::vector<std::pair<std::string, int>> added;    // added tokens matched on raw text
    int unk_id = -1;
    int cls_id = -1, sep_id = -1, pad_id = -1, mask_id = -1;  // TokenizerInfo (tokenizer_wrapper.rs:45-92)
    int tpl_cls = -1, tpl_sep = -1;                    // TemplateProcessing "[CLS] $A [SEP]" ids

    // ---- Unicode tables (data/bert_uncased_unicode.bin) ----------------------
    std::vector<uint16_t> upage;
    std::vector<uint32_t> uentry;
    std::vector<uint8_t> upool;
    std::vector<uint32_t> ubmp;
    std::vector<uint8_t> upfx;   // Unigram: longest plain piece under each hashed 4-byte prefix  // per BMP code point: device-format entry, WordPiece ISO id (wp_iso_ids)

    // ---- device image of the vocabulary ------------------------------------
    std::vector<VSlot> slots;
    std::vector<uint8_t> vpool;
    std::vector<int32_t> ascii_id;  // id of the one-byte word b (ISO ASCII fast path)
    uint32_t slot_mask = 0;
    int maxlen_first = 0, maxlen_cont = 0;
    std::vector<uint8_t> wp_lens[2];  // WordPiece: distinct payload lengths <= LW_MAX (non-"##", "##")
    bool wp_long_pieces = false;      // a payload longer than LW_MAX exists
    uint32_t opener = 0;
    int max_special_len = 0;

    // ---- byte-level BPE (gpt2) ---------------------------------------------
    int eos_id = -1;                       // <|endoftext|> (TokenizerInfo.eos)
    std::vector<uint16_t> byte_id;         // byte -> id of its byte-level symbol
    std::vector<MSlot> mslots;             // (left, right) -> (rank, merged)
    uint32_t mslot_mask = 0;
    std::vector<uint16_t> gpage;           // data/gpt2_classes.bin
    std::vector<uint8_t> gblock;
    size_t word_table_entries = 0;

    // ---- Unigram (t5) ------------------------------------------------------
    std::vector<double> uscore;            // id -> score
    std::vector<float> uscore32;           // ... nearest f32
    std::vector<int8_t> uscore_adj;        // ... f64 ulps from it (-1, 0, 1)
    std::vector<uint16_t> wres;            // word-table results of > 1 id
    std::vector<VSlot> wslots;             // word table (UC_WORD), apart from the pieces in `slots`
    uint32_t wslot_mask = 0;
    std::vector<uint16_t> tpage;           // data/t5_graphemes.bin
    std::vector<uint8_t> tblock;
    std::vector<uint16_t> cpage;           // device per-code-point table (page -> block)
    std::vector<uint32_t> cent;            // blocks of 256 (x, y) entries: see common.hpp CP_*
    std::vector<uint32_t> trie;            // Precompiled charsmap double array
    std::vector<uint8_t> tnorm;            // ... normalized strings
    double unk_score = 0.0;
    int maxlen_piece = 0;                  // longest vocab piece (bytes)
    int max_word = 0;                      // longest word-table word (bytes)
    int tpl_eos = -1;                      // TemplateProcessing "$A </s>" id
    std::vector<int> extra_ids;            // <extra_id_0..99>
};

// Unigram: ids of Viterbi("▁" + word) for an ASCII word, host side (same code
// as the kernels, unigram.hpp); used to precompute the word table.
std::vector<int> unigram_encode_word(const HostTokenizer &t, const uint8_t *w, size_t n);

// HF BPE::merge_word over raw bytes (byte-level symbols), host side: used to
// precompute the word table; same semantics as the device merge loop.
std::vector<int> bpe_encode_bytes(const HostTokenizer &t, const uint8_t *s, size_t n);

// Loads a HF tokenizer.json (WordPiece model with BertNormalizer +
// BertPreTokenizer, as bert-base-uncased) or a WordPiece vocab.txt, plus the
// Unicode table from data_dir.  Throws std::runtime_error with a message on
// anything unsupported.
void load_tokenizer(const std::string &path, const std::string &data_dir, HostTokenizer &out);

// Slot hash of a vocab piece (payload bytes, cont = "##"-prefixed); the
// kernels compute the same function (tokenize_wordpiece.hip: hinit/hmix/hfinal).
uint32_t piece_hash(const uint8_t *payload, size_t n, uint32_t cont);

}  // namespace sdl
