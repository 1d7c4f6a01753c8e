// assets.hpp -- tokenizer assets on the host, packed for the device.
#pragma once

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "common.hpp"

namespace sdl {

struct HostTokenizer {
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

    // ---- device image of the vocabulary ------------------------------------
    std::vector<VSlot> slots;
    std::vector<uint8_t> vpool;
    uint32_t slot_mask = 0;
    int maxlen_first = 0, maxlen_cont = 0;
    uint32_t opener = 0;
    int max_special_len = 0;
};

// Loads a HF tokenizer.json (WordPiece model with BertNormalizer +
// BertPreTokenizer, as bert-base-uncased) or a WordPiece vocab.txt, plus the
// Unicode table from data_dir.  Throws std::runtime_error with a message on
// anything unsupported.
void load_tokenizer(const std::string &path, const std::string &data_dir, HostTokenizer &out);

uint64_t fnv1a(const uint8_t *p, size_t n, uint64_t h = FNV_BASIS);

}  // namespace sdl
