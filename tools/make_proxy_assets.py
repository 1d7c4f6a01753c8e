#!/usr/bin/env python3
"""Build the offline *proxy* bert-base-uncased tokenizer asset.

The reference loads `bert-base-uncased` from the HF hub at start-up
(`rust/src/tokenizer/tokenizer_holder.rs:64-82`, name at
`rust/src/tasks/masking/masking_cases.rs:51`).  There is no network and no vocab
file on disk, so this script trains a WordPiece vocabulary of the real size
(30,522) with the real special-id layout:

    [PAD]=0  [unused0..98]=1..99  [UNK]=100  [CLS]=101  [SEP]=102  [MASK]=103
    [unused99..993]=104..998     learned pieces 999..30521

using the HF `tokenizers` trainers (same project as the crate the reference
pins, `tokenizers 0.13.1`, `rust/Cargo.lock`).  The corpus is the reference's
own fixture (`data/test.json.gz`) plus English docstrings harvested from the
locally installed Python packages, so the vocabulary has a realistic
distribution of whole words and `##` continuation pieces.

Outputs (committed):
  streaming_data_loader_amd/assets/bert_proxy/vocab.txt
  streaming_data_loader_amd/assets/bert_proxy/tokenizer.json

Run once in the build container; the GPU box only reads the committed files.
"""
import ast
import gzip
import json
import os
import random
import sys

from tokenizers import Tokenizer, models, normalizers, pre_tokenizers, processors, trainers
from tokenizers.implementations import BertWordPieceTokenizer

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "streaming_data_loader_amd", "assets", "bert_proxy")
FIXTURE = os.path.join(REPO, "tests", "golden", "test_records.jsonl")

VOCAB_SIZE = 30522
N_RESERVED = 999  # [PAD] + 99 unused + 4 specials + 895 unused  (ids 0..998)


def fixture_texts():
    with open(FIXTURE, "r", encoding="utf-8") as f:
        return [json.loads(l)["text"] for l in f]


def docstring_corpus(limit_bytes=40 << 20, seed=7):
    roots = ["/usr/local/lib/python3.10/dist-packages", "/usr/lib/python3.10"]
    files = []
    for root in roots:
        for dp, _, fns in os.walk(root):
            for fn in fns:
                if fn.endswith(".py"):
                    files.append(os.path.join(dp, fn))
    files.sort()
    random.Random(seed).shuffle(files)
    out, total = [], 0
    for path in files:
        try:
            with open(path, "r", encoding="utf-8") as f:
                tree = ast.parse(f.read())
        except Exception:
            continue
        for node in ast.walk(tree):
            if isinstance(node, (ast.FunctionDef, ast.ClassDef, ast.Module, ast.AsyncFunctionDef)):
                d = ast.get_docstring(node)
                if d and len(d) > 40 and sum(c.isascii() for c in d) > 0.98 * len(d):
                    out.append(d)
                    total += len(d)
        if total >= limit_bytes:
            break
    return out


def main():
    os.makedirs(OUT, exist_ok=True)
    texts = fixture_texts() * 40 + docstring_corpus()
    specials = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    # WordPieceTrainer is a BPE trainer with the "##" continuation prefix; the
    # BPE trainer is used directly so that the piece length can be capped like
    # the real vocabulary's (its longest pieces are < 20 bytes).
    tok = Tokenizer(models.BPE(unk_token="[UNK]", continuing_subword_prefix="##"))
    tok.normalizer = normalizers.BertNormalizer(lowercase=True)
    tok.pre_tokenizer = pre_tokenizers.BertPreTokenizer()
    n_learn = VOCAB_SIZE - N_RESERVED
    trainer = trainers.BpeTrainer(vocab_size=n_learn + len(specials) + 64,
                                  special_tokens=specials, min_frequency=2,
                                  limit_alphabet=1000, continuing_subword_prefix="##",
                                  max_token_length=18)
    tok.train_from_iterator(texts, trainer)
    learned = sorted(tok.get_vocab().items(), key=lambda kv: kv[1])
    learned = [t for t, _ in learned if t not in specials][:n_learn]
    assert len(learned) == n_learn, len(learned)
    vocab = ["[PAD]"] + [f"[unused{i}]" for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    vocab += [f"[unused{i}]" for i in range(99, 99 + N_RESERVED - len(vocab))]
    assert len(vocab) == N_RESERVED
    vocab += learned
    assert len(vocab) == VOCAB_SIZE and len(set(vocab)) == VOCAB_SIZE
    vpath = os.path.join(OUT, "vocab.txt")
    with open(vpath, "w", encoding="utf-8") as f:
        f.write("\n".join(vocab) + "\n")
    bert = BertWordPieceTokenizer(vpath, lowercase=True, clean_text=True,
                                  handle_chinese_chars=True, strip_accents=None)
    bert.save(os.path.join(OUT, "tokenizer.json"))
    t = Tokenizer.from_file(os.path.join(OUT, "tokenizer.json"))
    for s, want in (("[PAD]", 0), ("[UNK]", 100), ("[CLS]", 101), ("[SEP]", 102), ("[MASK]", 103)):
        assert t.token_to_id(s) == want, (s, t.token_to_id(s))
    enc = t.encode(fixture_texts()[0])
    print("vocab", len(vocab), "first ids", enc.ids[:12], file=sys.stderr)


if __name__ == "__main__":
    main()
