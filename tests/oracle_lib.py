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
ORACLE_SO = os.environ.get("ORACLE_SO") or os.path.join(ORACLE_DIR, "build", "liboracle.so")
VOCAB_TXT = os.path.join(REPO, "streaming_data_loader_amd", "assets", "bert_proxy", "vocab.txt")
UNICODE_BIN = os.path.join(REPO, "streaming_data_loader_amd", "data", "bert_uncased_unicode.bin")
GPT2_JSON = os.path.join(REPO, "streaming_data_loader_amd", "assets", "gpt2_proxy", "tokenizer.json")
GPT2_CLASSES = os.path.join(REPO, "streaming_data_loader_amd", "data", "gpt2_classes.bin")
T5_JSON = os.path.join(REPO, "streaming_data_loader_amd", "assets", "t5_proxy", "tokenizer.json")
T5_GRAPHEMES = os.path.join(REPO, "streaming_data_loader_amd", "data", "t5_graphemes.bin")

_lib = None


def build():
    if os.environ.get("ORACLE_SO"):  # a prebuilt variant (the sanitizer build of test_inflate_fuzz.py)
        return ORACLE_SO
    srcs = [os.path.join(ORACLE_DIR, f) for f in os.listdir(ORACLE_DIR) if f.endswith((".c", ".h"))]
    if not os.path.exists(ORACLE_SO) or os.path.getmtime(ORACLE_SO) < max(os.path.getmtime(f) for f in srcs):
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
        L.orc_chacha_block.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, vp]
        L.orc_stdrng_first_u64.restype = ctypes.c_uint64
        L.orc_stdrng_first_u64.argtypes = [vp]
        L.orc_rand_positions.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, vp]
        L.orc_mlm_key.restype = ctypes.c_uint32
        L.orc_mlm_key.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]
        L.orc_batcher_new.restype = vp
        L.orc_batcher_new.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_uint64]
        L.orc_batcher_push.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t, vp, vp]
        L.orc_batcher_flush.argtypes = [vp, vp, vp]
        L.orc_batcher_free.argtypes = [vp]
        L.orc_batcher_set_next_record.argtypes = [vp, ctypes.c_uint64]
        L.orc_batcher_set_rng_mode.argtypes = [vp, ctypes.c_int]
        L.orc_encoder_size.restype = ctypes.c_size_t
        L.orc_encoder_bert.argtypes = [vp, vp]
        L.orc_encoder_bert.restype = None
        L.orc_cfg_default.argtypes = [ctypes.POINTER(OrcCfg), ctypes.c_int]
        L.orc_cfg_default.restype = None
        L.orc_batcher_create.restype = vp
        L.orc_batcher_create.argtypes = [vp, ctypes.POINTER(OrcCfg)]
        L.orc_batcher_push_ex.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t, vp, ctypes.c_size_t,
                                          ctypes.POINTER(OrcOut)]
        L.orc_batcher_flush_ex.argtypes = [vp, ctypes.POINTER(OrcOut)]
        L.orc_gpt2_load.restype = vp
        L.orc_gpt2_load.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.orc_gpt2_free.argtypes = [vp]
        L.orc_gpt2_encode.restype = ctypes.c_long
        L.orc_gpt2_encode.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t, vp, ctypes.c_size_t]
        L.orc_gpt2_eos.argtypes = [vp]
        L.orc_encoder_gpt2.argtypes = [vp, vp]
        L.orc_encoder_gpt2.restype = None
        L.orc_t5_load.restype = vp
        L.orc_t5_load.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.orc_t5_free.argtypes = [vp]
        for f in ("orc_t5_encode", "orc_t5_normalize", "orc_t5_graphemes"):
            getattr(L, f).restype = ctypes.c_long
            getattr(L, f).argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t, vp, ctypes.c_size_t]
        L.orc_t5_eos.argtypes = [vp]
        L.orc_t5_special_id.argtypes = [vp, ctypes.c_char_p]
        L.orc_encoder_t5.argtypes = [vp, vp]
        L.orc_encoder_t5.restype = None
        L.orc_span_table.argtypes = [ctypes.c_double, ctypes.c_int, vp, vp, vp, ctypes.c_int]
        L.orc_span_table.restype = None
        L.orc_batcher_span_errors.argtypes = [vp]
        L.orc_pickle_dataset.restype = ctypes.c_size_t
        L.orc_pickle_dataset.argtypes = [ctypes.c_int] * 5 + [vp] * 5 + [vp, ctypes.c_size_t]
        L.orc_batcher_span_errors.restype = ctypes.c_uint64
        L.orc_normal_pcg32.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, vp]
        L.orc_normal_pcg32.restype = None
        L.orc_normal_row.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, vp]
        L.orc_normal_row.restype = None
        L.orc_json_number.restype = ctypes.c_int
        L.orc_json_number.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_double)]
        _lib = L
    return _lib


class OrcCfg(ctypes.Structure):
    _fields_ = [("task", ctypes.c_int32), ("B", ctypes.c_int32), ("S", ctypes.c_int32), ("chunk", ctypes.c_int32),
                ("min_ids", ctypes.c_int32), ("mask_length", ctypes.c_int32), ("mask_id", ctypes.c_int32),
                ("number_labels", ctypes.c_int32), ("avg_span_gap", ctypes.c_double),
                ("avg_span_size", ctypes.c_double), ("seed", ctypes.c_uint64), ("rng_mode", ctypes.c_int32)]


class OrcOut(ctypes.Structure):
    _fields_ = [("ids", ctypes.c_void_p), ("am", ctypes.c_void_p), ("tt", ctypes.c_void_p),
                ("lab", ctypes.c_void_p), ("f32", ctypes.c_void_p), ("rows", ctypes.c_int32)]


MLM, CLM, SPAN, MULTI_LABEL = 0, 1, 2, 3
SINGLE_CLASS = 4


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

    def push_into(self, b):
        """push() without copying the batch out (the planes stay in self.buf);
        returns rows of a finished batch or 0."""
        rows = ctypes.c_int()
        if lib().orc_batcher_push(self.h, b, len(b), self.buf.ctypes.data, ctypes.byref(rows)):
            return rows.value
        return 0

    def flush(self):
        rows = ctypes.c_int()
        if lib().orc_batcher_flush(self.h, self.buf.ctypes.data, ctypes.byref(rows)):
            return self.buf.copy(), rows.value
        return None

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_batcher_free(self.h)
            self.h = None


class Gpt2Tok:
    """The gpt2 byte-level BPE restatement (oracle/orc_bpe.c)."""

    def __init__(self, path=GPT2_JSON, classes=GPT2_CLASSES):
        self.h = lib().orc_gpt2_load(path.encode(), classes.encode())
        if not self.h:
            raise RuntimeError("oracle gpt2 tokenizer load failed")
        self.eos = lib().orc_gpt2_eos(self.h)

    def encode(self, text):
        b = text.encode("utf-8") if isinstance(text, str) else bytes(text)
        out = np.zeros(len(b) + 8, np.uint32)
        n = lib().orc_gpt2_encode(self.h, b, len(b), out.ctypes.data, out.size)
        return out[:n].tolist()


class T5Tok:
    """The t5 Precompiled + Unigram restatement (oracle/orc_unigram.c)."""

    def __init__(self, path=T5_JSON, graphemes=T5_GRAPHEMES):
        self.h = lib().orc_t5_load(path.encode(), graphemes.encode())
        if not self.h:
            raise RuntimeError("oracle t5 tokenizer load failed")
        self.eos = lib().orc_t5_eos(self.h)

    def _call(self, fn, text, cap_per_byte, dtype):
        b = text.encode("utf-8") if isinstance(text, str) else bytes(text)
        cap = cap_per_byte * len(b) + 8
        while True:
            out = np.zeros(cap, dtype)
            n = fn(self.h, b, len(b), out.ctypes.data, out.size)
            if n <= cap:
                return out[:n]
            cap = n

    def encode(self, text):
        return self._call(lib().orc_t5_encode, text, 2, np.uint32).tolist()

    def normalize(self, text):
        return self._call(lib().orc_t5_normalize, text, 4, np.uint8).tobytes().decode("utf-8")

    def grapheme_starts(self, text):
        return self._call(lib().orc_t5_graphemes, text, 1, np.uint32).tolist()

    def special_id(self, s):
        return lib().orc_t5_special_id(self.h, s.encode())


def span_table(avg, lo, cap=32):
    kmin = ctypes.c_int32()
    n = ctypes.c_int32()
    thr = np.zeros(cap, np.uint32)
    lib().orc_span_table(avg, lo, ctypes.byref(kmin), ctypes.byref(n), thr.ctypes.data, cap)
    return kmin.value, thr[:n.value].tolist()


class Encoder:
    """An orc_encoder (tokenizer + encode_mask framing) in owned storage."""

    def __init__(self, kind="bert", tok=None):
        self.buf = ctypes.create_string_buffer(lib().orc_encoder_size())
        self.tok = tok
        if kind == "bert":
            lib().orc_encoder_bert(tok.h, self.buf)
        elif kind == "gpt2":
            lib().orc_encoder_gpt2(tok.h, self.buf)
        elif kind == "t5":
            lib().orc_encoder_t5(tok.h, self.buf)
        else:
            raise ValueError(kind)


class OracleBatcherEx:
    """Generic oracle Batcher (oracle/orc_batcher.c): GenTokenizer for
    mlm/clm, SimpleBatcher for multi-label.  push/flush return a dict of the
    batch planes (copies) or None."""

    def __init__(self, encoder, task, B, S, mask_length=None, mask_id=103, number_labels=9, seed=0,
                 chunk=None, min_ids=None, avg_span_gap=16.0, avg_span_size=2.0, rng_mode=0):
        c = OrcCfg()
        lib().orc_cfg_default(ctypes.byref(c), task)
        c.B, c.S, c.mask_id, c.number_labels, c.seed = B, S, mask_id, number_labels, seed
        c.rng_mode = rng_mode
        c.avg_span_gap, c.avg_span_size = avg_span_gap, avg_span_size
        c.mask_length = int(np.float32(S) * np.float32(0.15)) if mask_length is None else mask_length
        if chunk is not None:
            c.chunk = 1 if chunk else 0
        if min_ids is not None:
            c.min_ids = min_ids
        self.enc, self.task, self.B, self.S, self.NL = encoder, task, B, S, number_labels
        self.h = lib().orc_batcher_create(encoder.buf, ctypes.byref(c))
        if not self.h:
            raise RuntimeError("oracle batcher config rejected")
        LW = S if task in (MLM, CLM) else S // 4 if task == SPAN else 1 if task == SINGLE_CLASS else 0
        self.planes = {"input_ids": np.zeros((B, S), np.int32), "attention_mask": np.zeros((B, S), np.int32),
                       "token_type_ids": np.zeros((B, S), np.int32), "labels": np.zeros((B, max(LW, 1)), np.int32),
                       "labels_f32": np.zeros((B, number_labels), np.float32)}
        p = self.planes
        self.out = OrcOut(p["input_ids"].ctypes.data, p["attention_mask"].ctypes.data,
                          p["token_type_ids"].ctypes.data, p["labels"].ctypes.data if LW else None,
                          p["labels_f32"].ctypes.data if task == MULTI_LABEL else None, 0)

    def set_next_record(self, r):
        lib().orc_batcher_set_next_record(self.h, r)

    def _result(self):
        d = {k: v.copy() for k, v in self.planes.items()}
        d["rows"] = self.out.rows
        return d

    def push(self, text, labels=None):
        b = text.encode("utf-8") if isinstance(text, str) else bytes(text)
        lab = None if labels is None else np.ascontiguousarray(labels, np.uint32)
        rc = lib().orc_batcher_push_ex(self.h, b, len(b), None if lab is None else lab.ctypes.data,
                                       0 if lab is None else lab.size, ctypes.byref(self.out))
        if rc < 0:
            raise ValueError("label index >= number_labels")
        return self._result() if rc == 1 else None

    def push_raw(self, b, labels=None):
        """push() of bytes without copying a finished batch out (timing)."""
        lab = None if labels is None else np.ascontiguousarray(labels, np.uint32)
        return lib().orc_batcher_push_ex(self.h, b, len(b), None if lab is None else lab.ctypes.data,
                                         0 if lab is None else lab.size, ctypes.byref(self.out))

    def flush(self):
        return self._result() if lib().orc_batcher_flush_ex(self.h, ctypes.byref(self.out)) == 1 else None

    def span_errors(self):
        return int(lib().orc_batcher_span_errors(self.h))

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_batcher_free(self.h)
            self.h = None


def oracle_rows(tok, texts, S, mask_length, mask_id=103, seed=0, B=64, first_record=0, rng_mode=0):
    """All rows the reference Batcher would produce for `texts`, in order
    (concatenation of every batch, flushing until the queue is empty)."""
    ob = OracleBatcher(tok, B, S, mask_length, mask_id, seed)
    ob.set_next_record(first_record)
    lib().orc_batcher_set_rng_mode(ob.h, rng_mode)
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


TASK_IDS = {"mlm": 0, "clm": 1, "span": 2, "multi-label": 3, "single-class": 4}


def pickle_dataset(task, B, S, LW, rows, input_ids, attention_mask, token_type_ids, labels):
    """serde_pickle::to_vec(&DataSet) bytes (oracle/orc_pickle.c).  Planes are
    numpy [B, S] int32 (labels [B, LW] int32, or float32 for multi-label)."""
    L = lib()
    arrs = [np.ascontiguousarray(a) if a is not None else None
            for a in (input_ids, attention_mask, token_type_ids, labels)]
    ptr = [a.ctypes.data if a is not None else None for a in arrs]
    f32 = task == "multi-label"
    args = [TASK_IDS[task], B, S, LW, rows, ptr[0], ptr[1], ptr[2], None if f32 else ptr[3], ptr[3] if f32 else None]
    n = L.orc_pickle_dataset(*args, None, 0)
    out = np.zeros(n, np.uint8)
    assert L.orc_pickle_dataset(*args, out.ctypes.data, n) == n
    return out.tobytes()


def gz_inflate(member):
    """oracle/orc_inflate.c: one gzip member -> (status, inflated bytes); status
    codes are the device's GZ_* codes (0 ok)."""
    L = lib()
    if not hasattr(L, "_gz_ready"):
        L.orc_gz_isize.restype = ctypes.c_uint32
        L.orc_gz_isize.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.orc_gz_inflate.restype = ctypes.c_int
        L.orc_gz_inflate.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.POINTER(ctypes.c_size_t)]
        L._gz_ready = True
    m = bytes(member)
    cap = L.orc_gz_isize(m, len(m)) if len(m) >= 18 else 0
    cap = min(cap, 1032 * len(m) + 64)  # DEFLATE expands at most ~1032:1 (the device's sizing bound)
    buf = ctypes.create_string_buffer(max(cap, 1))
    got = ctypes.c_size_t(0)
    st = L.orc_gz_inflate(m, len(m), buf, cap, ctypes.byref(got))
    return st, buf.raw[:got.value]


def json_number(text):
    """A JSON number as serde_json 1.0.87 parses it into an f64 (oracle/orc_json.c)."""
    b = text.encode() if isinstance(text, str) else bytes(text)
    out = ctypes.c_double()
    if lib().orc_json_number(b, len(b), ctypes.byref(out)):
        raise ValueError(f"not a JSON number: {b!r}")
    return out.value
