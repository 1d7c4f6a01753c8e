"""Pin the t5 path to the reference's own t5 known-answer vector.

`/root/reference/python/test_t5.py:3-7`: t5-small encodes
"I am here to save the day. The dog is done with the food." (add_special_tokens=True) as
[27, 183, 270, 12, 1097, 8, 239, 5, 37, 1782, 19, 612, 28, 8, 542, 5, 1].  Every word is
one piece, so the ids fix 14 pieces (and </s>) at their t5-small indices.
`tests/golden/make_t5_kat_vocab.py` builds the t5 proxy tokenizer with those pieces moved
to those ids (the rest of the 32,100-entry vocabulary and the Precompiled charsmap are the
proxy's).  Reproducing the 17 ids through it pins the added-token split, the Precompiled
normalizer on this text, WhitespaceSplit, Metaspace's "▁" prefix, the Unigram Viterbi's
choice against the full vocabulary and the `$A </s>` template to the reference's output --
here for the C oracle and `tokenizers`; tests/test_gpu_t5_kat.py for the HIP path."""
import os
import sys

import pytest

import oracle_lib

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLDEN)
import make_t5_kat_vocab as kat  # noqa: E402


@pytest.fixture(scope="module")
def kat_tokenizer(tmp_path_factory):
    d = tmp_path_factory.mktemp("t5_kat")
    import json
    path = os.path.join(str(d), "tokenizer.json")
    with open(path, "w", encoding="utf-8") as f:
        json.dump(kat.build(), f, ensure_ascii=False)
    return path


def test_kat_vector_is_the_references():
    # /root/reference/python/test_t5.py:7 (the comment under the call)
    assert kat.KAT_IDS == [27, 183, 270, 12, 1097, 8, 239, 5, 37, 1782, 19, 612, 28, 8, 542, 5, 1]
    assert kat.KAT_TEXT == "I am here to save the day. The dog is done with the food."
    assert sorted(set(kat.KAT_IDS) - {1}) == sorted(kat.KAT_PIECES)


def test_kat_vocabulary_layout(kat_tokenizer):
    import json
    with open(kat_tokenizer, encoding="utf-8") as f:
        v = json.load(f)["model"]["vocab"]
    assert len(v) == 32100 and len({p for p, _ in v}) == 32100
    for i, p in kat.KAT_PIECES.items():
        assert v[i][0] == p
    assert [v[i][0] for i in (0, 1, 2)] == ["<pad>", "</s>", "<unk>"]
    assert v[32099][0] == "<extra_id_0>" and v[32000][0] == "<extra_id_99>"


def test_oracle_reproduces_the_kat(kat_tokenizer):
    tok = oracle_lib.T5Tok(kat_tokenizer)
    assert tok.encode(kat.KAT_TEXT) == kat.KAT_IDS


def test_tokenizers_reproduces_the_kat(kat_tokenizer):
    tokenizers = pytest.importorskip("tokenizers")
    t = tokenizers.Tokenizer.from_file(kat_tokenizer)
    assert t.encode(kat.KAT_TEXT).ids == kat.KAT_IDS


def test_kat_tokenizer_is_accepted_by_the_product_host_check(native_lib, kat_tokenizer):
    from streaming_data_loader_amd import native
    info = native.tokenizer_info(kat_tokenizer)
    assert info.kind == 2 and info.eos_id == 1 and info.unk_id == 2 and info.vocab_size == 32100
