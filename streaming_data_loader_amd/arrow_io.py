"""Arrow record input for the multi-label task.

Reference: MultiArrowGenerator (rust/src/tasks/multi_label/multi_arrow.rs:11-41)
turns each Arrow row into a SimpleTransport {text: sentence, label:
Label::Multi(labels)} one `slice(0,1)` at a time, and ArrowTransfer
(rust/src/provider/arrow_transfer.rs:48-118) streams the record batches.

Here the same schema (`sentence: utf8`, `labels: list<int64>`) is read with
pyarrow and a whole record batch becomes the Batcher's text arena without a
per-row copy: the utf8 column's value buffer IS the arena and its int32 offsets
become the uint64 record offsets; the list column's offsets/values become the
Label::Multi index arrays.  `MultiArrowGenerator.get_data` keeps the
reference's per-row form for callers that want SimpleTransport objects.
"""
from dataclasses import dataclass
from typing import Iterator

import numpy as np

from .batcher import Label, SimpleData, SimpleTransport


def _pa():
    import pyarrow as pa  # host-side dependency of the Arrow provider only
    return pa


def read_stream(source) -> Iterator["pyarrow.RecordBatch"]:  # noqa: F821
    """Record batches of an Arrow IPC stream (path, bytes or file-like)."""
    pa = _pa()
    if isinstance(source, (bytes, bytearray, memoryview)):
        source = pa.BufferReader(source)
    with pa.ipc.open_stream(source) as r:
        for b in r:
            yield b


class MultiArrowGenerator:
    """ArrowGenerator for multi-label rows (multi_arrow.rs:11-41)."""

    def __init__(self, schema):
        self.t = schema.get_field_index("sentence")
        self.l = schema.get_field_index("labels")
        if self.t < 0 or self.l < 0:
            raise KeyError("schema needs `sentence` and `labels` columns")  # reference: unwrap() panics

    def get_data(self, batch, row: int = 0) -> SimpleTransport:
        text = batch.column(self.t)[row].as_py()
        labels = [int(x) for x in batch.column(self.l)[row].as_py()]
        return SimpleTransport(SimpleData(text, None), Label(multi=labels))


class SingleClassArrowGenerator:
    """ArrowGenerator for single-class rows (single_class/single_arrow.rs:11-39):
    `text` utf8 + `label` int64 -> SimpleTransport with Label::Single(label as u32)."""

    def __init__(self, schema):
        self.t = schema.get_field_index("text")
        self.l = schema.get_field_index("label")
        if self.t < 0 or self.l < 0:
            raise KeyError("schema needs `text` and `label` columns")  # reference: unwrap() panics

    def get_data(self, batch, row: int = 0) -> SimpleTransport:
        text = batch.column(self.t)[row].as_py()
        label = int(batch.column(self.l)[row].as_py()) & 0xFFFFFFFF  # `as u32`
        return SimpleTransport(SimpleData(text, None), Label(single=label))


@dataclass
class ArrowArena:
    arena: np.ndarray          # uint8, the utf8 value bytes (+16 B pad)
    offsets: np.ndarray        # uint64 [n+1], offsets[0] = 0
    labels: np.ndarray         # uint32 Label::Multi indices
    label_offsets: np.ndarray  # uint64 [n+1]

    @property
    def n_records(self):
        return self.offsets.size - 1


def _int_offsets(buf, offset, n, width):
    dt = np.int32 if width == 4 else np.int64
    return np.frombuffer(buf, dt, count=offset + n + 1, offset=0)[offset:offset + n + 1]


def arena_from_batch(batch, text_col="sentence", label_col="labels") -> ArrowArena:
    """One record batch -> text arena + offsets + label arrays, read straight
    from the Arrow buffers (nulls are taken as empty text / no labels)."""
    pa = _pa()
    t = batch.column(batch.schema.get_field_index(text_col))
    if t.type not in (pa.utf8(), pa.large_utf8()):
        raise TypeError(f"{text_col} must be utf8, got {t.type}")
    n = len(t)
    w = 8 if t.type == pa.large_utf8() else 4
    _, obuf, vbuf = t.buffers()
    o = _int_offsets(obuf, t.offset, n, w).astype(np.int64)
    if t.null_count:
        valid = np.asarray(t.is_valid())
        lens = np.where(valid, np.diff(o), 0)
        starts = o[:-1]
        pieces = [np.frombuffer(vbuf, np.uint8, count=int(l), offset=int(s)) for s, l in zip(starts, lens)]
        body = np.concatenate(pieces) if pieces else np.zeros(0, np.uint8)
        offs = np.zeros(n + 1, np.uint64)
        np.cumsum(lens, out=offs[1:])
    else:
        base, end = int(o[0]), int(o[-1])
        body = np.frombuffer(vbuf, np.uint8, count=end - base, offset=base) if end > base else np.zeros(0, np.uint8)
        offs = (o - base).astype(np.uint64)
    arena = np.concatenate([body, np.zeros(16, np.uint8)])

    lc = batch.column(batch.schema.get_field_index(label_col))
    if pa.types.is_integer(lc.type):  # SingleClassArrowGenerator: one label per row, `as u32`
        if lc.null_count:
            raise ValueError("null label")  # Int64Array::value of a null slot is not a label
        vals = (np.asarray(lc, np.int64) & 0xFFFFFFFF).astype(np.uint32)
        return ArrowArena(arena, offs, vals, np.arange(n + 1, dtype=np.uint64))
    if not pa.types.is_list(lc.type) and not pa.types.is_large_list(lc.type):
        raise TypeError(f"{label_col} must be list<int64>, got {lc.type}")
    lo = np.asarray(lc.offsets, dtype=np.int64)
    if lc.null_count:
        valid = np.asarray(lc.is_valid())
        cnt = np.where(valid, np.diff(lo), 0)
        vals = np.concatenate([np.asarray(lc.values[int(s):int(s + c)], np.int64)
                               for s, c in zip(lo[:-1], cnt)] or [np.zeros(0, np.int64)])
        loffs = np.zeros(n + 1, np.uint64)
        np.cumsum(cnt, out=loffs[1:])
    else:
        vals = np.asarray(lc.values, np.int64)[int(lo[0]):int(lo[-1])]
        loffs = (lo - lo[0]).astype(np.uint64)
    if vals.size and (vals.min() < 0 or vals.max() > 0xFFFFFFFF):
        raise ValueError("label index out of u32 range")  # `e.unwrap() as u32` in the reference
    return ArrowArena(arena, offs, vals.astype(np.uint32), loffs)
