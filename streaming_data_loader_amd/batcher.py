"""Python mirror of the reference Batcher interface over the HIP library.

Same names, argument meaning and error behaviour as the reference's Rust:
  BatchConfig            rust/src/batcher.rs:11-23
  Batcher (trait)        rust/src/batcher.rs:26-31
  create_batch (driver)  rust/src/batcher.rs:33-77
  GenTokenizer           rust/src/tasks/gen_batcher.rs:12-98
  DataSetConfig          rust/src/datasets/dataset_config.rs:7-16
  ModelType / TaskType   rust/src/config.rs:20-62
  ProviderChannel        rust/src/provider/mod.rs:21-25
  masking cases          rust/src/tasks/masking/masking_cases.rs:34-94
  SimpleBatcher          rust/src/models/simple_batcher.rs:8-53
  SimpleTransport/Label  rust/src/models/simple_transport.rs, simple_label.rs
Every record's tokenize + mask runs in libsdl_batcher.so on the GPU.
"""
import ctypes
import enum
from dataclasses import dataclass, field
from typing import Optional, Union

import numpy as np

from . import native


# ---- configuration (serde structs of the reference) ----------------------------
@dataclass
class BatchConfig:
    batch_size: int
    sequence_length: int


@dataclass
class Mask:
    mask_length: int
    mask: int = 103


@dataclass
class Gpt:
    pass


@dataclass
class Span:
    avg_span_gap: float = 16.0
    avg_span_size: float = 2.0


@dataclass
class MultiLabel:
    number_labels: int = 9


@dataclass
class SingleClass:
    """DataSetConfig::SingleClass (dataset_config.rs; single_cases.rs: Imdb)."""


DataSetConfig = Union[Mask, Gpt, Span, MultiLabel, SingleClass]


class ModelType(enum.Enum):
    Bert = "bert"
    Roberta = "roberta"
    Gpt2 = "gpt2"
    T5 = "t5"


class TaskType(enum.Enum):
    Mlm = "mlm"
    Clm = "clm"
    Span = "span"
    MultiLabel = "multi-label"
    SingleClass = "single-class"


@dataclass
class TokenizerConfig:
    """TokenizerInternalConfig: the reference names a hub tokenizer
    (HuggingFace("bert-base-uncased")); offline, `path` is its tokenizer.json."""
    path: str = native.BERT_PROXY_TOKENIZER


@dataclass
class TrainingConfig:
    model_config: ModelType
    tokenizer: TokenizerConfig
    batch: BatchConfig
    dataset_config: DataSetConfig
    seed: int = 0
    device: int = 0
    # 0: the Philox contract; 1: the reference's own draws on a
    # per-row StdRng::from_seed(seed | record | chunk) -- rand 0.8.5 shuffle
    # for MLM masks, rand_distr 0.4.3 StandardNormal for span gaps / sizes
    # (INTEGRATION.md "Provable parity")
    rng_mode: int = 0


def get_mask_length(sequence_length: int) -> int:
    """masking_cases.rs:34-36: (sequence_length as f32 * 0.15) as usize."""
    return int(np.float32(sequence_length) * np.float32(0.15))


def get_case(task: TaskType, test: bool, sequence_length: int = 128, batch_size: Optional[int] = None,
             seed: int = 0, rng_mode: int = 0) -> TrainingConfig:
    """masking_cases::get_case: B=4096 (test: 1), S=128 unless overridden."""
    b = batch_size if batch_size is not None else (1 if test else 4096)
    batch = BatchConfig(b, sequence_length)
    if task == TaskType.Mlm:
        return TrainingConfig(ModelType.Bert, TokenizerConfig(), batch, Mask(get_mask_length(sequence_length), 103),
                              seed, rng_mode=rng_mode)
    if task == TaskType.Clm:  # masking_cases.rs:66: gpt2
        return TrainingConfig(ModelType.Gpt2, TokenizerConfig(native.GPT2_PROXY_TOKENIZER), batch, Gpt(), seed,
                              rng_mode=rng_mode)
    if task == TaskType.Span:  # masking_cases.rs:78-90: t5-small, Span{16.0, 2.0}
        return TrainingConfig(ModelType.T5, TokenizerConfig(native.T5_PROXY_TOKENIZER), batch, Span(16.0, 2.0), seed,
                              rng_mode=rng_mode)
    return TrainingConfig(ModelType.Bert, TokenizerConfig(), BatchConfig(2048 if batch_size is None else b,
                                                                        sequence_length), MultiLabel(9), seed,
                          rng_mode=rng_mode)


# ---- channel messages --------------------------------------------------------
class ProviderChannel:
    @dataclass
    class Info:
        value: object

    @dataclass
    class Data:
        value: object

    class Complete:
        pass


# ---- DataSet -------------------------------------------------------------------
@dataclass
class DataSet:
    """One batch; `to_dict()` is the reference's Serialize view
    (bert_data.rs:106-145, gpt_data.rs:53-62, t5_data.rs:235-249).  `labels` is
    int32 [B, S] for mlm/clm, int32 [B, S/4] for span and float32
    [B, number_labels] for multi-label."""
    kind: str
    rows: int
    input_ids: np.ndarray
    attention_mask: np.ndarray
    labels: np.ndarray
    token_type_ids: Optional[np.ndarray] = None

    def to_dict(self):
        if self.kind == "bert-single":
            # DataSetConfig::SingleClass: "label" is Vec<u32>, one per filled row (bert_data.rs:118-121)
            return {"input_ids": self.input_ids, "attention_mask": self.attention_mask,
                    "token_type_ids": self.token_type_ids, "label": self.labels[:self.rows, 0]}
        if self.kind == "bert":
            # BertData.label is pushed per row: the list has `index` entries
            # (Vec<i32> for Mask, Vec<f32> for MultiLabel)
            return {"input_ids": self.input_ids, "attention_mask": self.attention_mask,
                    "token_type_ids": self.token_type_ids, "labels": self.labels[:self.rows]}
        return {"input_ids": self.input_ids, "attention_mask": self.attention_mask, "labels": self.labels}


def _native_config(batch_config, dataset_config, chunk, seed, device, first_record, rng_mode):
    """sdl_config for a ModelType/DataSetConfig pair (config.rs:43-62) -> (config, batch kind)."""
    if isinstance(dataset_config, Mask):
        task, kind = native.SDL_TASK_MLM, "bert"
    elif isinstance(dataset_config, Gpt):
        task, kind = native.SDL_TASK_CLM, "gpt2"
    elif isinstance(dataset_config, Span):
        task, kind = native.SDL_TASK_SPAN, "t5"
    elif isinstance(dataset_config, SingleClass):
        task, kind = native.SDL_TASK_SINGLE_CLASS, "bert-single"
    else:
        task, kind = native.SDL_TASK_MULTI_LABEL, "bert"
    c = native.default_config(task)
    c.batch_size, c.sequence_length = batch_config.batch_size, batch_config.sequence_length
    c.chunk = 1 if chunk else 0
    if isinstance(dataset_config, Mask):
        c.mask_length, c.mask_id = dataset_config.mask_length, dataset_config.mask
    if isinstance(dataset_config, Span):
        c.avg_span_gap, c.avg_span_size = dataset_config.avg_span_gap, dataset_config.avg_span_size
    if isinstance(dataset_config, MultiLabel):
        c.number_labels = dataset_config.number_labels
    c.seed, c.device, c.first_record, c.rng_mode = seed, device, first_record, rng_mode
    return c, kind


class _BatchOwner:
    """Keeps a finished sdl_batch alive while numpy views of its planes exist;
    the batch's pinned block returns to the handle's pool when the last view
    goes (sdl_batch_release)."""
    __slots__ = ("b", "_release", "_byref")

    def __init__(self, b):
        self.b = b
        self._release = native.load().sdl_batch_release  # bound now (teardown-safe)
        self._byref = ctypes.byref

    def __del__(self):
        try:
            self._release(self._byref(self.b))
        except Exception:  # interpreter shutdown
            pass


def _dataset_from(b: native.Batch, kind: str) -> DataSet:
    """Zero-copy: the DataSet's arrays are views of the batch's pinned planes
    (the D2H wrote them there directly)."""
    b = native.Batch.from_buffer_copy(b)  # callers reuse their sdl_batch struct
    B, S, LW = b.batch_size, b.sequence_length, b.label_width
    owner = _BatchOwner(b)

    def arr(ptr, n, cols, ctype, dtype):
        buf = (ctype * (n * cols)).from_address(ctypes.cast(ptr, ctypes.c_void_p).value)
        buf._owner = owner
        return np.frombuffer(buf, dtype=dtype).reshape(n, cols)

    i32 = (ctypes.c_int32, np.int32)
    labels = arr(b.labels_f32, B, LW, ctypes.c_float, np.float32) if bool(b.labels_f32) else arr(b.labels, B, LW, *i32)
    return DataSet(kind=kind, rows=b.rows, input_ids=arr(b.input_ids, B, S, *i32),
                   attention_mask=arr(b.attention_mask, B, S, *i32), labels=labels,
                   token_type_ids=arr(b.token_type_ids, B, S, *i32) if bool(b.token_type_ids) else None)


# ---- SimpleTransport (models/simple_transport.rs, simple_label.rs) ----------------
@dataclass
class SimpleData:
    text: str
    alt_text: Optional[str] = None


@dataclass
class Label:
    """simple_label::Label: Multi(Vec<u32>) or Single(u32) reach the GPU Batcher."""
    multi: Optional[list] = None
    single: Optional[int] = None


@dataclass
class SimpleTransport:
    data: SimpleData
    label: Optional[Label] = None


def _pack_labels(label_lists):
    """Label::Multi indices of many records -> (uint32 values, uint64 offsets)."""
    offs = np.zeros(len(label_lists) + 1, np.uint64)
    np.cumsum([len(x) for x in label_lists], out=offs[1:])
    vals = np.fromiter((int(v) for x in label_lists for v in x), np.uint32, count=int(offs[-1]))
    return vals, offs


# ---- Batcher -------------------------------------------------------------------
class Batcher:
    """trait Batcher (batcher.rs:26-31)."""

    def create_sync_batch(self, data):
        raise NotImplementedError

    def get_working_batch(self):
        raise NotImplementedError


class _NativeBatcher(Batcher):
    """One sdl_batcher handle (include/sdl_batcher.h)."""

    def __init__(self, model_type: ModelType, batch_config: BatchConfig, dataset_config: DataSetConfig,
                 tokenizer: TokenizerConfig, chunk: bool = True, seed: int = 0, device: int = 0,
                 first_record: int = 0, rng_mode: int = 0):
        L = native.load()
        c, self.kind = _native_config(batch_config, dataset_config, chunk, seed, device, first_record, rng_mode)
        h = ctypes.c_void_p()
        native.check(L.sdl_batcher_create(ctypes.byref(c), tokenizer.path.encode(), native.DATA_DIR.encode(),
                                          ctypes.byref(h)))
        self._h = h
        self._destroy = L.sdl_batcher_destroy  # bound now: close() may run at interpreter teardown
        native.track(self)
        self.batch_config = batch_config
        self.dataset_config = dataset_config

    @classmethod
    def from_config(cls, cfg: TrainingConfig, chunk: bool = True):
        """masking_runner::create_generator (masking_runner.rs:55-62)."""
        return cls(cfg.model_config, cfg.batch, cfg.dataset_config, cfg.tokenizer, chunk, cfg.seed, cfg.device,
                   rng_mode=cfg.rng_mode)

    def close(self):
        if getattr(self, "_h", None):
            self._destroy(self._h)
            self._h = None

    __del__ = close

    def _push(self, raw: bytes, labels=None) -> Optional[DataSet]:
        b = native.Batch()
        lab = None if labels is None else np.ascontiguousarray(labels, np.uint32)
        got = native.check(native.load().sdl_batcher_push(self._h, raw, len(raw),
                                                          None if lab is None else lab.ctypes.data,
                                                          0 if lab is None else lab.size, ctypes.byref(b)))
        return _dataset_from(b, self.kind) if got else None

    def push_arena(self, arena, offsets, labels=None, label_offsets=None):
        """sdl_batcher_push_many over a host arena (uint8) + uint64 offsets
        (+ uint32 label values / uint64 label offsets); returns the batches
        the same sequence of create_sync_batch calls would have emitted."""
        arena = np.ascontiguousarray(arena, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        n = ctypes.c_size_t()
        lv = None if labels is None else np.ascontiguousarray(labels, np.uint32)
        lo = None if label_offsets is None else np.ascontiguousarray(label_offsets, np.uint64)
        native.check(native.load().sdl_batcher_push_many(
            self._h, arena.ctypes.data, offsets.ctypes.data, offsets.size - 1,
            None if lv is None or lv.size == 0 else lv.ctypes.data, None if lo is None else lo.ctypes.data,
            ctypes.byref(n)))
        out = []
        b = native.Batch()
        while native.check(native.load().sdl_batcher_next(self._h, ctypes.byref(b))):
            out.append(_dataset_from(b, self.kind))
        return out

    def get_working_batch(self) -> Optional[DataSet]:
        b = native.Batch()
        got = native.check(native.load().sdl_batcher_flush(self._h, ctypes.byref(b)))
        return _dataset_from(b, self.kind) if got else None


class GenTokenizer(_NativeBatcher):
    """GenTokenizer (gen_batcher.rs:12-98): S = String, T = DataSet.  Each call
    tokenizes + masks on the GPU; the emission cadence is the reference's (at
    most one batch per create_sync_batch, one batch on get_working_batch)."""

    def create_sync_batch(self, data: str) -> Optional[DataSet]:
        return self._push(data.encode("utf-8") if isinstance(data, str) else bytes(data))

    def create_sync_batches(self, texts):
        """create_sync_batch over many records in one device pass; returns the
        batches the same sequence of calls would have emitted, in order."""
        blobs = [t.encode("utf-8") if isinstance(t, str) else t for t in texts]
        offs = np.zeros(len(blobs) + 1, np.uint64)
        np.cumsum(np.fromiter(map(len, blobs), np.uint64, len(blobs)), out=offs[1:])
        arena = np.frombuffer(b"".join(blobs), np.uint8)  # the C side stages (and pads) it
        return self.push_arena(arena, offs)


class SimpleBatcher(_NativeBatcher):
    """SimpleBatcher (models/simple_batcher.rs:8-53): S = SimpleTransport,
    T = DataSet, for DataSetConfig::MultiLabel.  One row per record (encode_mask
    framing, truncated at S, no <64 filter); the batch is returned by the
    create_sync_batch call that fills it; get_working_batch always returns the
    current (possibly empty) batch and starts a new one."""

    def __init__(self, model_type: ModelType, dataset_config: DataSetConfig, batch_config: BatchConfig,
                 tokenizer: TokenizerConfig, seed: int = 0, device: int = 0, rng_mode: int = 0):
        if not isinstance(dataset_config, (MultiLabel, SingleClass)):
            raise ValueError("SimpleBatcher on the GPU path supports DataSetConfig::MultiLabel / SingleClass")
        # (these tasks draw nothing at random; rng_mode is accepted and checked like everywhere)
        super().__init__(model_type, batch_config, dataset_config, tokenizer, False, seed, device, rng_mode=rng_mode)

    @classmethod
    def from_config(cls, cfg: TrainingConfig):
        """single_class::runner::create_generator (single_class/runner.rs:40-49)."""
        return cls(cfg.model_config, cfg.dataset_config, cfg.batch, cfg.tokenizer, cfg.seed, cfg.device,
                   rng_mode=cfg.rng_mode)

    def create_sync_batch(self, data: SimpleTransport) -> Optional[DataSet]:
        text = data.data.text
        raw = text.encode("utf-8") if isinstance(text, str) else bytes(text)
        if isinstance(self.dataset_config, SingleClass):
            if data.label is None or data.label.single is None:
                # the reference's label.map(push) would skip the label and misalign the
                # label list; SingleClassArrowGenerator always yields Some(Label::Single)
                raise ValueError("single-class records carry exactly one Label::Single")
            return self._push(raw, [data.label.single])
        if data.label is None or data.label.multi is None:
            raise ValueError("Label Type Not Supported")  # bert_data.rs:75 panics
        return self._push(raw, data.label.multi)

    def create_sync_batches(self, items):
        """create_sync_batch over many SimpleTransport records in one device pass."""
        blobs = [t.data.text.encode("utf-8") if isinstance(t.data.text, str) else bytes(t.data.text) for t in items]
        offs = np.zeros(len(blobs) + 1, np.uint64)
        np.cumsum([len(x) for x in blobs], out=offs[1:])
        arena = np.frombuffer(b"".join(blobs) + b"\0" * 16, np.uint8)
        single = isinstance(self.dataset_config, SingleClass)
        vals, loffs = _pack_labels([[t.label.single] if single else t.label.multi for t in items])
        return self.push_arena(arena, offs, vals, loffs)

    def push_arrow(self, record_batch, text_col=None, label_col=None):
        """create_sync_batch for every row of an Arrow record batch with the
        MultiArrowGenerator schema (sentence, labels: list<int64>) or the
        SingleClassArrowGenerator one (text, label: int64), fed from the column
        buffers directly."""
        from .arrow_io import arena_from_batch
        single = isinstance(self.dataset_config, SingleClass)
        a = arena_from_batch(record_batch, text_col or ("text" if single else "sentence"),
                             label_col or ("label" if single else "labels"))
        return self.push_arena(a.arena, a.offsets, a.labels, a.label_offsets)


def create_batch(rx, tx, batcher: Batcher):
    """batcher::create_batch (batcher.rs:33-77): Info passes through, Data is
    batched, Complete flushes one working batch then forwards Complete.
    rx/tx are queue-like (get()/put()); a None message ends the loop."""
    while True:
        msg = rx.get()
        if msg is None:
            break
        if isinstance(msg, ProviderChannel.Info):
            tx.put(msg)
        elif isinstance(msg, ProviderChannel.Complete) or msg is ProviderChannel.Complete:
            cur = batcher.get_working_batch()
            if cur is not None:
                tx.put(ProviderChannel.Data(cur))
            tx.put(ProviderChannel.Complete())
            break
        elif isinstance(msg, ProviderChannel.Data):
            batch = batcher.create_sync_batch(msg.value)
            if batch is not None:
                tx.put(ProviderChannel.Data(batch))


def _record_bytes(x):
    if isinstance(x, SimpleTransport):
        x = x.data.text
    return len(x) if isinstance(x, (bytes, bytearray)) else len(x) * 4 if isinstance(x, str) else 0


_NOTHING = object()


def create_batch_drained(rx, tx, batcher: _NativeBatcher, max_bytes: int = 64 << 20, max_records: int = 1 << 20):
    """batcher::create_batch (batcher.rs:33-77) for the GPU Batcher: every
    ProviderChannel::Data already waiting in `rx` (up to max_bytes of text /
    max_records) is drained and handed to the device in ONE
    sdl_batcher_push_many call, instead of one device round trip per record.

    The Data sequence sent to `tx` is the per-record loop's, message for
    message: push_many queues exactly the batches the same sequence of
    create_sync_batch calls would emit (at most one per record, in order, the
    handle keeping GenTokenizer's/SimpleBatcher's queue across calls), they
    are sent before the message that ended the drain, Info passes through in
    stream order, and Complete flushes one get_working_batch() then forwards
    Complete.  rx needs get() (blocking) and get_nowait() (raising
    queue.Empty); a None message ends the loop like a closed channel."""
    import queue
    pending, size = [], 0

    def flush():
        nonlocal pending, size
        if pending:
            for ds in batcher.create_sync_batches(pending):
                tx.put(ProviderChannel.Data(ds))
        pending, size = [], 0

    while True:
        msg = rx.get()
        # drain what is already waiting (never block with records pending)
        while isinstance(msg, ProviderChannel.Data):
            pending.append(msg.value)
            size += _record_bytes(msg.value)
            if size >= max_bytes or len(pending) >= max_records:
                flush()
            try:
                msg = rx.get_nowait()
            except queue.Empty:
                msg = _NOTHING
        flush()
        if msg is _NOTHING:
            continue
        if msg is None:
            break
        if isinstance(msg, ProviderChannel.Info):
            tx.put(msg)
        elif isinstance(msg, ProviderChannel.Complete) or msg is ProviderChannel.Complete:
            cur = batcher.get_working_batch()
            if cur is not None:
                tx.put(ProviderChannel.Data(cur))
            tx.put(ProviderChannel.Complete())
            break


class ShardedGenTokenizer:
    """One record stream over several GPUs (sdl_multi_*): every push is cut
    into byte-balanced contiguous record ranges (sdl_shard_records), one per device; each
    shard runs on its own handle, HIP stream and host thread, concurrently.  Shard k's
    batches are those a GenTokenizer (gen_batcher.rs:65-98) over its record range emits, and
    masks are keyed by the global record index, so every row equals the row one handle would
    give over the whole stream -- N reference Batchers on disjoint shards, no collective.
    `devices` may repeat a device (tests drive several shards on one GPU)."""

    def __init__(self, model_type: ModelType, batch_config: BatchConfig, dataset_config: DataSetConfig,
                 tokenizer: TokenizerConfig, devices, chunk: bool = True, seed: int = 0, first_record: int = 0,
                 rng_mode: int = 0):
        L = native.load()
        c, self.kind = _native_config(batch_config, dataset_config, chunk, seed, 0, first_record, rng_mode)
        devs = (ctypes.c_int32 * len(devices))(*devices)
        m = ctypes.c_void_p()
        native.check(L.sdl_multi_create(ctypes.byref(c), tokenizer.path.encode(), native.DATA_DIR.encode(), devs,
                                        len(devices), ctypes.byref(m)))
        self._m = m
        self._destroy = L.sdl_multi_destroy
        self.n = len(devices)
        self.batch_config = batch_config
        native.track(self)

    def close(self):
        if getattr(self, "_m", None):
            self._destroy(self._m)
            self._m = None

    __del__ = close

    def handle(self, k):
        """Shard k's sdl_batcher handle (owned by this object)."""
        return native.load().sdl_multi_handle(self._m, k)

    def push_arena(self, arena, offsets, labels=None, label_offsets=None):
        """sdl_multi_push_many: returns, per shard, the batches it emitted (in order).
        labels / label_offsets (uint32 values, uint64 offsets into them) for the
        multi-label and single-class tasks, as sdl_batcher_push_many takes them."""
        arena = np.ascontiguousarray(arena, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        lv = None if labels is None else np.ascontiguousarray(labels, np.uint32)
        lo = None if label_offsets is None else np.ascontiguousarray(label_offsets, np.uint64)
        n = (ctypes.c_size_t * self.n)()
        L = native.load()
        native.check(L.sdl_multi_push_many(self._m, arena.ctypes.data, offsets.ctypes.data, offsets.size - 1,
                                           None if lv is None or lv.size == 0 else lv.ctypes.data,
                                           None if lo is None else lo.ctypes.data, n))
        out = []
        for k in range(self.n):
            got, b, h = [], native.Batch(), self.handle(k)
            while native.check(L.sdl_batcher_next(h, ctypes.byref(b))):
                got.append(_dataset_from(b, self.kind))
            out.append(got)
        return out

    def create_sync_batches(self, texts):
        blobs = [t.encode("utf-8") if isinstance(t, str) else t for t in texts]
        offs = np.zeros(len(blobs) + 1, np.uint64)
        np.cumsum(np.fromiter(map(len, blobs), np.uint64, len(blobs)), out=offs[1:])
        return self.push_arena(np.frombuffer(b"".join(blobs), np.uint8), offs)

    def get_working_batch(self, k) -> Optional[DataSet]:
        """Shard k's Batcher::get_working_batch (its flushed partial batch)."""
        b = native.Batch()
        got = native.check(native.load().sdl_batcher_flush(self.handle(k), ctypes.byref(b)))
        return _dataset_from(b, self.kind) if got else None
