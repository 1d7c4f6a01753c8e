#!/usr/bin/env python3
"""Build the offline *proxy* gpt2 tokenizer asset.

The reference loads `gpt2` from the HF hub (`Tokenizer::from_pretrained`,
rust/src/tokenizer/tokenizer_holder.rs:64-82; name at
rust/src/tasks/masking/masking_cases.rs:66).  Offline, this trains a byte-level
BPE of the real size and layout with the HF `tokenizers` trainer (same project
as the crate the reference pins, tokenizers 0.13.1):

    ByteLevel pre-tokenizer (GPT-2 regex, add_prefix_space=false)
    BPE: 50,256 learned/base tokens (the 256 byte symbols first) + 50,000-ish merges
    <|endoftext|> = 50256 (added special token)
    ByteLevel post-processor / decoder

on the reference fixture (data/test.json.gz) plus English docstrings of the
locally installed Python packages (tools/make_proxy_assets.py corpus).

Output (committed): streaming_data_loader_amd/assets/gpt2_proxy/tokenizer.json
"""
import os
import sys

from tokenizers import Tokenizer, decoders, models, pre_tokenizers, processors, trainers

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_proxy_assets import docstring_corpus, fixture_texts  # noqa: E402

REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "streaming_data_loader_amd", "assets", "gpt2_proxy")
VOCAB = 50257


def main():
    os.makedirs(OUT, exist_ok=True)
    texts = fixture_texts() * 40 + docstring_corpus()
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=True)
    tok.decoder = decoders.ByteLevel()
    tok.post_processor = processors.ByteLevel(trim_offsets=False)
    trainer = trainers.BpeTrainer(vocab_size=VOCAB - 1, min_frequency=2, show_progress=False,
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet(), special_tokens=[])
    tok.train_from_iterator(texts, trainer)
    assert tok.get_vocab_size() == VOCAB - 1, tok.get_vocab_size()
    tok.add_special_tokens(["<|endoftext|>"])
    assert tok.token_to_id("<|endoftext|>") == VOCAB - 1
    path = os.path.join(OUT, "tokenizer.json")
    tok.save(path)
    t = Tokenizer.from_file(path)
    enc = t.encode(fixture_texts()[0])
    print("vocab", t.get_vocab_size(), "first ids", enc.ids[:12], file=sys.stderr)


if __name__ == "__main__":
    main()
