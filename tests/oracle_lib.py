"""ctypes access to the CPU oracle (oracle/sdl_oracle.c) -- test infrastructure.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this,
and only as the checker / CPU baseline, never as the product path.
"""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "liboracle.so")
VOCAB_TXT = os.path.join(REPO, "streaming_data_loader_amd", "assets", "bert_proxy", "vocab.txt")
UNICODE_BIN = os.path.join(REPO, "streaming_data_loader_amd", "data", "bert_uncased_unicode.bin")

_lib = None


def build():
    src = os.path.join(ORACLE_DIR, "sdl_oracle.c")
    if not os.path.exists(ORACLE_SO) or os.path.getmtime(ORACLE_SO) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    return ORACLE_SO


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(ORACLE_SO)
        vp = ctypes.c_void_p
        L.orc_tok_load.restype = vp
        L.orc_tok_load.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.orc_tok_free.argtypes = [vp]
        L.orc_bert_encode.restype = ctypes.c_long
        L.orc_bert_encode.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t, vp, ctypes.c_size_t]
        L.orc_mlm_key.restype = ctypes.c_uint32
        L.orc_mlm_key.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]
        L.orc_batcher_new.restype = vp
        L.orc_batcher_new.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_uint64]
        L.orc_batcher_push.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t, vp, vp]
        L.orc_batcher_flush.argtypes = [vp, vp, vp]
        L.orc_batcher_free.argtypes = [vp]
        L.orc_batcher_set_next_record.argtypes = [vp, ctypes.c_uint64]
        _lib = L
    return _lib


class Tok:
    def __init__(self, vocab=VOCAB_TXT, unicode_bin=UNICODE_BIN):
        self.h = lib().orc_tok_load(vocab.encode(), unicode_bin.encode())
        if not self.h:
            raise RuntimeError("oracle tokenizer load failed")

    def encode(self, text):
        b = text.encode("utf-8") if isinstance(text, str) else bytes(text)
        out = np.zeros(len(b) + 8, np.uint32)
        n = lib().orc_bert_encode(self.h, b, len(b), out.ctypes.data, out.size)
        return out[:n].tolist()


class OracleBatcher:
    """GenTokenizer(chunk=true) + BertData(Mask) on the CPU (the checker)."""

    def __init__(self, tok, B, S, mask_length, mask_id=103, seed=0):
        self.B, self.S = B, S
        self.h = lib().orc_batcher_new(tok.h, 0, B, S, mask_length, mask_id, seed)
        if not self.h:
            raise RuntimeError("oracle batcher config rejected")
        self.buf = np.zeros((4, B, S), np.int32)

    def set_next_record(self, r):
        lib().orc_batcher_set_next_record(self.h, r)

    def push(self, text):
        b = text.encode("utf-8") if isinstance(text, str) else bytes(text)
        rows = ctypes.c_int()
        if lib().orc_batcher_push(self.h, b, len(b), self.buf.ctypes.data, ctypes.byref(rows)):
            return self.buf.copy(), rows.value
        return None

    def flush(self):
        rows = ctypes.c_int()
        if lib().orc_batcher_flush(self.h, self.buf.ctypes.data, ctypes.byref(rows)):
            return self.buf.copy(), rows.value
        return None

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_batcher_free(self.h)
            self.h = None


def oracle_rows(tok, texts, S, mask_length, mask_id=103, seed=0, B=64, first_record=0):
    """All rows the reference Batcher would produce for `texts`, in order
    (concatenation of every batch, flushing until the queue is empty)."""
    ob = OracleBatcher(tok, B, S, mask_length, mask_id, seed)
    ob.set_next_record(first_record)
    planes = []
    for t in texts:
        r = ob.push(t)
        if r is not None:
            planes.append(r[0][:, :r[1]])
    while True:
        r = ob.flush()
        if r is None:
            break
        planes.append(r[0][:, :r[1]])
    if not planes:
        return np.zeros((4, 0, S), np.int32)
    return np.concatenate(planes, axis=1)
