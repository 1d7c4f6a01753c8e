"""Device-resident bulk path: a text arena already in HBM -> packed [rows, S]
planes in HBM, through sdl_process_device (the measured hot path).

PyTorch is used only to hold device memory and streams.
"""
import ctypes

import numpy as np

from . import native


class _CudaView:
    """__cuda_array_interface__ (v3) of device memory the library owns: what
    torch.as_tensor / cupy / numba take without a copy."""

    def __init__(self, ptr, shape, typestr, stream=None):
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": typestr, "data": (int(ptr), False),
                                         "version": 3}
        if stream:  # the producer's stream: the consumer orders its reads after it
            self.__cuda_array_interface__["stream"] = int(stream)


class DeviceResult:
    def __init__(self, handle, rows_struct, n_records, S, B=None, device=0, stream=0):
        self.h = handle
        self.r = rows_struct
        self.n_records = n_records
        self.S = S
        self.B = B
        self.device = device
        self.stream = stream  # the caller's stream the work was queued on (0: the handle's own)

    def rows(self):
        v = np.zeros(1, np.uint32)
        native.d2h(self.h, v, self.r.d_rows, 4)
        return int(v[0])

    def tokens(self):
        v = np.zeros(1, np.uint32)
        native.d2h(self.h, v, self.r.d_tokens, 4)
        return int(v[0])

    def record_rows(self):
        v = np.zeros(self.n_records, np.uint32)
        native.d2h(self.h, v, self.r.d_record_rows, 4 * self.n_records)
        return v

    def label_errors(self):
        """Multi-label: Label::Multi indices >= number_labels that were skipped;
        span: label / sentinel writes past their bounds (the reference panics)."""
        if not self.r.d_label_errors:
            return 0
        v = np.zeros(1, np.uint32)
        native.d2h(self.h, v, self.r.d_label_errors, 4)
        return int(v[0])

    def tokenize_errors(self):
        """t5 tokenizer: capacity flags (include/sdl_batcher.h), 0 = ok."""
        if not self.r.d_tokenize_errors:
            return 0
        v = np.zeros(1, np.uint32)
        native.d2h(self.h, v, self.r.d_tokenize_errors, 4)
        return int(v[0])

    def planes(self, n_rows=None):
        """(input_ids, attention_mask, token_type_ids|None, labels) as numpy [n, S]
        (labels: int32 [n, S] for mlm/clm, float32 [n, number_labels] for multi-label)."""
        n = self.rows() if n_rows is None else n_rows
        S, LW = self.S, self.r.label_width

        def get(ptr, w, dt=np.int32):
            a = np.zeros((n, w), dt)
            if ptr:
                native.d2h(self.h, a, ptr, a.nbytes)
                return a
            return None

        lab = get(self.r.labels_f32, LW, np.float32) if self.r.labels_f32 else get(self.r.labels, LW)
        return (get(self.r.input_ids, S), get(self.r.attention_mask, S), get(self.r.token_type_ids, S), lab)

    def tensors(self, n_rows=None, device=None):
        """The planes as zero-copy torch tensors on the device, keyed as the
        reference's DataSet (input_ids, attention_mask, token_type_ids when the
        task has them, labels: int32 [n, S], float32 [n, number_labels] for
        multi-label).  Views of the handle's buffers: valid until its next call."""
        import torch
        # rows() synchronizes the handle's stream (work queued without a caller stream); work
        # on a caller's stream is ordered through the interface's "stream" key instead
        rows = self.rows()
        n = rows if n_rows is None else n_rows
        S, LW = self.S, self.r.label_width
        dev = device if device is not None else torch.device("cuda", self.device)
        out = {}
        for key, ptr, w, ts in (("input_ids", self.r.input_ids, S, "<i4"),
                                ("attention_mask", self.r.attention_mask, S, "<i4"),
                                ("token_type_ids", self.r.token_type_ids, S, "<i4"),
                                ("labels", self.r.labels_f32 or self.r.labels, LW, "<f4" if self.r.labels_f32 else "<i4")):
            if ptr and n > 0:
                out[key] = torch.as_tensor(_CudaView(ptr, (n, w), ts, self.stream), device=dev)
        return out

    def batches(self, n_rows=None, device=None):
        """Consumer side without the pickle (a zero-copy tensor
        frame instead of serde_pickle -> pickle.loads, external_dataset.py:52):
        every batch as a dict of [B, ...] device tensor views plus its "rows"
        (the last batch holds the rest; its pad rows keep the initial values)."""
        if not self.B:
            raise ValueError("batches() needs the batch size (DeviceBatcher results carry it)")
        n = self.rows() if n_rows is None else n_rows
        nb = -(-n // self.B)
        full = self.tensors(nb * self.B, device)
        return [dict({k: v[b * self.B:(b + 1) * self.B] for k, v in full.items()}, rows=min(self.B, n - b * self.B))
                for b in range(nb)]


class DeviceFrames:
    """Transport frames on the device (sdl_pickle_frames_device): frame f is
    d_frames[f*frame_bytes : f*frame_bytes + size(f)], the bytes
    serde_pickle::to_vec(&DataSet) gives the socket (zmq_transmit.rs:71)."""

    def __init__(self, handle, fr):
        self.h = handle
        self.f = fr

    def __len__(self):
        return int(self.f.n_frames)

    def to_host(self):
        """All frames as one uint8 array (D2H copy)."""
        a = np.zeros(int(self.f.total_bytes), np.uint8)
        return native.d2h(self.h, a, self.f.d_frames, a.nbytes)

    def frames(self):
        """List of bytes objects, one per batch."""
        a = self.to_host().tobytes()
        n, F = len(self), int(self.f.frame_bytes)
        return [a[i * F:(i * F + (F if i < n - 1 else int(self.f.last_frame_bytes)))] for i in range(n)]


class DeviceBatcher:
    """Owns one sdl_batcher handle used through sdl_process_device."""

    def __init__(self, task=native.SDL_TASK_MLM, batch_size=256, sequence_length=512, mask_length=None,
                 mask_id=103, seed=0, device=0, tokenizer=native.BERT_PROXY_TOKENIZER, chunk=True, min_ids=None,
                 number_labels=9, avg_span_gap=16.0, avg_span_size=2.0, rng_mode=0):
        L = native.load()
        c = native.default_config(task)
        c.batch_size, c.sequence_length = batch_size, sequence_length
        c.mask_length = int(np.float32(sequence_length) * np.float32(0.15)) if mask_length is None else mask_length
        c.mask_id, c.seed, c.device, c.chunk = mask_id, seed, device, 1 if chunk else 0
        c.number_labels = number_labels
        c.rng_mode = rng_mode
        c.avg_span_gap, c.avg_span_size = avg_span_gap, avg_span_size
        if min_ids is not None:
            c.min_ids = min_ids
        self.cfg = c
        h = ctypes.c_void_p()
        native.check(L.sdl_batcher_create(ctypes.byref(c), tokenizer.encode(), native.DATA_DIR.encode(),
                                          ctypes.byref(h)))
        self._h = h
        self._destroy = L.sdl_batcher_destroy  # bound now: close() may run at interpreter teardown
        native.track(self)

    def close(self):
        if getattr(self, "_h", None):
            self._destroy(self._h)
            self._h = None

    __del__ = close

    def set_profiling(self, on=True):
        native.check(native.load().sdl_set_profiling(self._h, 1 if on else 0))

    def stage_times(self):
        names = (ctypes.c_char_p * 16)()
        ms = (ctypes.c_float * 16)()
        n = native.check(native.load().sdl_stage_times(self._h, names, ms, 16))
        return {names[i].decode(): float(ms[i]) for i in range(n)}

    def process(self, text_ptr, text_len, offsets_ptr, n_records, first_record=0, stream=0):
        """Pointers are device addresses (ints), e.g. tensor.data_ptr()."""
        out = native.DeviceRows()
        native.check(native.load().sdl_process_device(self._h, ctypes.c_void_p(text_ptr), text_len,
                                                      ctypes.c_void_p(offsets_ptr), n_records, first_record,
                                                      ctypes.c_void_p(stream or None), ctypes.byref(out)))
        return DeviceResult(self._h, out, n_records, self.cfg.sequence_length, self.cfg.batch_size, self.cfg.device,
                            stream)

    def process_labels(self, text_ptr, text_len, offsets_ptr, n_records, labels_ptr, label_offsets_ptr,
                       first_record=0, stream=0):
        """Multi-label task: Label::Multi indices per record in device memory."""
        out = native.DeviceRows()
        native.check(native.load().sdl_process_device_labels(
            self._h, ctypes.c_void_p(text_ptr), text_len, ctypes.c_void_p(offsets_ptr), n_records,
            ctypes.c_void_p(labels_ptr or None), ctypes.c_void_p(label_offsets_ptr or None), first_record,
            ctypes.c_void_p(stream or None), ctypes.byref(out)))
        return DeviceResult(self._h, out, n_records, self.cfg.sequence_length, self.cfg.batch_size, self.cfg.device,
                            stream)

    def json_text(self, jsonl_ptr, jsonl_len, stream=0):
        """The provider's JsonText filter on the device (sdl_json_text_device):
        a 16-B aligned device buffer of JSON lines -> the `text` records as a
        device arena + offsets owned by this handle (native.JsonText)."""
        out = native.JsonText()
        native.check(native.load().sdl_json_text_device(self._h, ctypes.c_void_p(jsonl_ptr), jsonl_len,
                                                        ctypes.c_void_p(stream or None), ctypes.byref(out)))
        return out

    def gzip_inflate(self, gz_ptr, gz_len, member_offsets_ptr, n_members, stream=0, check=True):
        """The provider's gzip inflate on the device (sdl_gzip_inflate_device):
        gzip members in a 16-B aligned device buffer -> their bytes back to back
        in a device arena owned by this handle (native.Inflated).  check=False
        returns (rc, Inflated) instead of raising on corrupt members."""
        out = native.Inflated()
        rc = native.load().sdl_gzip_inflate_device(self._h, ctypes.c_void_p(gz_ptr), gz_len,
                                                   ctypes.c_void_p(member_offsets_ptr), n_members,
                                                   ctypes.c_void_p(stream or None), ctypes.byref(out))
        if check:
            native.check(rc)
            return out
        return rc, out

    def gzip_inflate_first(self, gz_ptr, gz_len, file_offsets_ptr, n_files, stream=0, check=True):
        """Reference-exact gzip (sdl_gzip_inflate_first_device): every range is a file and only its
        first member is inflated, as async-compression's GzipDecoder reads a file."""
        out = native.Inflated()
        rc = native.load().sdl_gzip_inflate_first_device(self._h, ctypes.c_void_p(gz_ptr), gz_len,
                                                         ctypes.c_void_p(file_offsets_ptr), n_files,
                                                         ctypes.c_void_p(stream or None), ctypes.byref(out))
        if check:
            native.check(rc)
            return out
        return rc, out

    def pickle_frames(self, result, n_rows=None, flush_partial=True, stream=0):
        """Transport step on the device: the batches of `result` (the last
        process*() call) as serde_pickle frames (DeviceFrames)."""
        n = result.rows() if n_rows is None else n_rows
        out = native.Frames()
        native.check(native.load().sdl_pickle_frames_device(self._h, ctypes.byref(result.r), n,
                                                            1 if flush_partial else 0,
                                                            ctypes.c_void_p(stream or None), ctypes.byref(out)))
        return DeviceFrames(self._h, out)

    def json_to_frames(self, jsonl, chunk_bytes=8 << 20, flush_partial=True, collect=True):
        """End to end, host to host (sdl_json_to_frames): JSON lines in host
        memory -> the serde_pickle frames of every batch, pipelined in chunks.
        Returns (list of frames or None, native.JsonFramesStats)."""
        buf = np.frombuffer(jsonl, np.uint8) if isinstance(jsonl, (bytes, bytearray)) else np.ascontiguousarray(jsonl)
        frames = [] if collect else None

        def sink(_user, ptr, n):
            frames.append(ctypes.string_at(ptr, n))
            return 0
        cb = native.FRAME_SINK(sink) if collect else ctypes.cast(None, native.FRAME_SINK)
        st = native.JsonFramesStats()
        native.check(native.load().sdl_json_to_frames(self._h, buf.ctypes.data if buf.size else None, buf.size,
                                                      chunk_bytes, 1 if flush_partial else 0, cb, None,
                                                      ctypes.byref(st)))
        return frames, st

    def process_tensors(self, text, offsets, first_record=0, stream=None):
        """text: uint8 cuda tensor; offsets: int64 cuda tensor of n_records+1 entries."""
        s = stream.cuda_stream if stream is not None else 0
        return self.process(text.data_ptr(), text.numel(), offsets.data_ptr(), offsets.numel() - 1, first_record, s)


def arena_from_texts(texts):
    """Host arena (uint8, padded) + uint64 offsets for a list of str/bytes."""
    blobs = [t.encode("utf-8") if isinstance(t, str) else bytes(t) for t in texts]
    offs = np.zeros(len(blobs) + 1, np.uint64)
    if blobs:
        np.cumsum([len(x) for x in blobs], out=offs[1:])
    arena = np.frombuffer(b"".join(blobs), np.uint8) if blobs else np.zeros(0, np.uint8)
    return arena, offs
