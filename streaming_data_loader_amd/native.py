"""ctypes binding of libsdl_batcher.so (include/sdl_batcher.h).

The product path is the HIP library only: if it is missing, or no GPU is
visible, these calls raise -- there is no CPU fallback.
"""
import atexit
import ctypes
import os
import weakref

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SDL_LIB") or os.path.join(PKG, "libsdl_batcher.so")
DATA_DIR = os.path.join(PKG, "data")
ASSETS = os.path.join(PKG, "assets")
BERT_PROXY_TOKENIZER = os.path.join(ASSETS, "bert_proxy", "tokenizer.json")
GPT2_PROXY_TOKENIZER = os.path.join(ASSETS, "gpt2_proxy", "tokenizer.json")
T5_PROXY_TOKENIZER = os.path.join(ASSETS, "t5_proxy", "tokenizer.json")

SDL_TASK_MLM, SDL_TASK_CLM, SDL_TASK_SPAN, SDL_TASK_MULTI_LABEL, SDL_TASK_SINGLE_CLASS = 0, 1, 2, 3, 4

# every symbol include/sdl_batcher.h declares
EXPORTS = [
    "sdl_config_default", "sdl_batcher_create", "sdl_batcher_destroy", "sdl_batcher_push",
    "sdl_batcher_push_many", "sdl_batcher_next", "sdl_batcher_flush", "sdl_batch_release",
    "sdl_process_device", "sdl_process_device_labels", "sdl_json_text_device", "sdl_pickle_frames_device", "sdl_device_to_host", "sdl_set_profiling", "sdl_stage_times",
    "sdl_tokenizer_info_get", "sdl_last_error", "sdl_abi_version", "sdl_json_to_frames",
    "sdl_gzip_inflate_device", "sdl_gzip_inflate_first_device", "sdl_gzip_split_members", "sdl_build_id",
    "sdl_shard_records", "sdl_multi_create", "sdl_multi_destroy", "sdl_multi_push_many", "sdl_multi_handle",
]


class SDLError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"sdl error {code}: {msg}")
        self.code = code


class Config(ctypes.Structure):
    _fields_ = [
        ("task", ctypes.c_int32), ("batch_size", ctypes.c_int32), ("sequence_length", ctypes.c_int32),
        ("chunk", ctypes.c_int32), ("min_ids", ctypes.c_int32), ("mask_length", ctypes.c_int32),
        ("mask_id", ctypes.c_int32), ("number_labels", ctypes.c_int32),
        ("avg_span_gap", ctypes.c_double), ("avg_span_size", ctypes.c_double),
        ("seed", ctypes.c_uint64), ("first_record", ctypes.c_uint64),
        ("device", ctypes.c_int32), ("rng_mode", ctypes.c_int32), ("reserved", ctypes.c_int32 * 6),
    ]


class Batch(ctypes.Structure):
    _fields_ = [
        ("rows", ctypes.c_int32), ("batch_size", ctypes.c_int32), ("sequence_length", ctypes.c_int32),
        ("label_width", ctypes.c_int32),
        ("input_ids", ctypes.POINTER(ctypes.c_int32)), ("attention_mask", ctypes.POINTER(ctypes.c_int32)),
        ("token_type_ids", ctypes.POINTER(ctypes.c_int32)), ("labels", ctypes.POINTER(ctypes.c_int32)),
        ("labels_f32", ctypes.POINTER(ctypes.c_float)), ("owner_", ctypes.c_void_p),
    ]


class DeviceRows(ctypes.Structure):
    _fields_ = [
        ("input_ids", ctypes.c_void_p), ("attention_mask", ctypes.c_void_p), ("token_type_ids", ctypes.c_void_p),
        ("labels", ctypes.c_void_p), ("labels_f32", ctypes.c_void_p), ("d_rows", ctypes.c_void_p),
        ("d_record_rows", ctypes.c_void_p), ("d_tokens", ctypes.c_void_p),
        ("rows_capacity", ctypes.c_uint64), ("label_width", ctypes.c_int32),
        ("d_label_errors", ctypes.c_void_p), ("d_tokenize_errors", ctypes.c_void_p),
    ]


class JsonText(ctypes.Structure):
    _fields_ = [
        ("d_text", ctypes.c_void_p), ("d_offsets", ctypes.c_void_p), ("n_records", ctypes.c_uint64),
        ("text_bytes", ctypes.c_uint64), ("n_lines", ctypes.c_uint64), ("n_invalid", ctypes.c_uint64),
    ]


class Frames(ctypes.Structure):
    _fields_ = [
        ("d_frames", ctypes.c_void_p), ("n_frames", ctypes.c_uint64), ("frame_bytes", ctypes.c_uint64),
        ("last_frame_bytes", ctypes.c_uint64), ("total_bytes", ctypes.c_uint64),
    ]


class JsonFramesStats(ctypes.Structure):
    _fields_ = [
        ("n_lines", ctypes.c_uint64), ("n_invalid", ctypes.c_uint64), ("n_records", ctypes.c_uint64),
        ("text_bytes", ctypes.c_uint64), ("n_rows", ctypes.c_uint64), ("n_frames", ctypes.c_uint64),
        ("frame_bytes", ctypes.c_uint64), ("n_chunks", ctypes.c_uint64), ("seconds", ctypes.c_double),
        ("host_wait", ctypes.c_double * 4),
    ]


class Inflated(ctypes.Structure):
    _fields_ = [
        ("d_out", ctypes.c_void_p), ("d_member_out", ctypes.c_void_p), ("d_status", ctypes.c_void_p),
        ("out_bytes", ctypes.c_uint64), ("n_members", ctypes.c_uint64), ("n_bad", ctypes.c_uint64),
    ]


# per-member status codes of sdl_gzip_inflate_device (csrc/kernels.hpp GZ_*)
GZ_OK, GZ_E_RANGE, GZ_E_TRUNC, GZ_E_HEADER, GZ_E_HCRC, GZ_E_BTYPE, GZ_E_STORED, GZ_E_CODES, GZ_E_CODE, \
    GZ_E_FAR, GZ_E_OVER, GZ_E_SIZE, GZ_E_TRAIL, GZ_E_CRC, GZ_E_STALL = range(15)
SDL_ERR_DATA = -8


FRAME_SINK = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8), ctypes.c_uint64)


class TokenizerInfo(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32), ("vocab_size", ctypes.c_int32), ("n_added", ctypes.c_int32),
        ("unk_id", ctypes.c_int32), ("eos_id", ctypes.c_int32), ("max_piece_bytes", ctypes.c_int32),
        ("word_table_entries", ctypes.c_uint64), ("reserved", ctypes.c_int32 * 6),
    ]


_lib = None
_live_handles = weakref.WeakSet()


def track(owner):
    """Objects holding an sdl_batcher handle: closed by atexit while the HIP runtime and this
    module are still alive (a __del__ at interpreter teardown would find both gone)."""
    _live_handles.add(owner)


@atexit.register
def _close_live_handles():
    for owner in list(_live_handles):
        try:
            owner.close()
        except Exception:
            pass


def load(path=LIB_PATH):
    """Loads the native library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise SDLError(-4, f"{path} missing: run `python -m streaming_data_loader_amd.build` (no CPU fallback)")
    # PyTorch-ROCm ships its own libamdhip64.so.7.  Load it first when torch is
    # installed so this library binds to the same HIP runtime (same soname)
    # instead of bringing a second runtime into the process.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    L = ctypes.CDLL(path)
    product = os.path.abspath(path) == os.path.join(PKG, "libsdl_batcher.so")
    if product or hasattr(L, "sdl_build_id"):  # (SDL_LIB diagnostic builds of older sources may lack it)
        L.sdl_build_id.restype = ctypes.c_char_p
        L.sdl_build_id.argtypes = []
    if product:
        # the product library must be built from the sources beside it
        # (build.py embeds their content hash): a stale prebuilt library fails here
        from . import build as _build
        got, want = L.sdl_build_id().decode(), _build.source_hash()
        if got != want:
            raise SDLError(-4, f"{path} was built from other sources (build id {got[:12]}, sources {want[:12]}): "
                               "rebuild with `python -m streaming_data_loader_amd.build`")
    vp, sz, u64, i32, i64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int
    L.sdl_config_default.argtypes = [ctypes.POINTER(Config), i32]
    L.sdl_config_default.restype = None
    L.sdl_batcher_create.argtypes = [ctypes.POINTER(Config), ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(vp)]
    L.sdl_batcher_destroy.argtypes = [vp]
    L.sdl_batcher_destroy.restype = None
    L.sdl_batcher_push.argtypes = [vp, ctypes.c_char_p, sz, vp, sz, ctypes.POINTER(Batch)]
    L.sdl_batcher_push_many.argtypes = [vp, vp, vp, sz, vp, vp, ctypes.POINTER(sz)]
    L.sdl_batcher_next.argtypes = [vp, ctypes.POINTER(Batch)]
    L.sdl_batcher_flush.argtypes = [vp, ctypes.POINTER(Batch)]
    L.sdl_batch_release.argtypes = [ctypes.POINTER(Batch)]
    L.sdl_batch_release.restype = None
    L.sdl_process_device.argtypes = [vp, vp, u64, vp, u64, u64, vp, ctypes.POINTER(DeviceRows)]
    L.sdl_process_device_labels.argtypes = [vp, vp, u64, vp, u64, vp, vp, u64, vp, ctypes.POINTER(DeviceRows)]
    L.sdl_device_to_host.argtypes = [vp, vp, vp, sz, vp]
    L.sdl_json_text_device.argtypes = [vp, vp, u64, vp, ctypes.POINTER(JsonText)]
    L.sdl_pickle_frames_device.argtypes = [vp, ctypes.POINTER(DeviceRows), u64, i64, vp, ctypes.POINTER(Frames)]
    L.sdl_json_to_frames.argtypes = [vp, vp, u64, u64, i64, FRAME_SINK, vp, ctypes.POINTER(JsonFramesStats)]
    L.sdl_json_to_frames.restype = i64
    L.sdl_gzip_inflate_device.argtypes = [vp, vp, u64, vp, u64, vp, ctypes.POINTER(Inflated)]
    L.sdl_gzip_inflate_device.restype = i64
    L.sdl_gzip_inflate_first_device.argtypes = [vp, vp, u64, vp, u64, vp, ctypes.POINTER(Inflated)]
    L.sdl_gzip_inflate_first_device.restype = i64
    L.sdl_gzip_split_members.argtypes = [vp, u64, vp, u64, ctypes.POINTER(u64)]
    L.sdl_gzip_split_members.restype = i64
    L.sdl_shard_records.argtypes = [vp, u64, ctypes.c_uint32, vp]
    L.sdl_shard_records.restype = i64
    L.sdl_multi_create.argtypes = [ctypes.POINTER(Config), ctypes.c_char_p, ctypes.c_char_p, vp, ctypes.c_uint32,
                                   ctypes.POINTER(vp)]
    L.sdl_multi_create.restype = i64
    L.sdl_multi_destroy.argtypes = [vp]
    L.sdl_multi_destroy.restype = None
    L.sdl_multi_push_many.argtypes = [vp, vp, vp, sz, vp, vp, vp]
    L.sdl_multi_push_many.restype = i64
    L.sdl_multi_handle.argtypes = [vp, ctypes.c_uint32]
    L.sdl_multi_handle.restype = vp
    L.sdl_set_profiling.argtypes = [vp, i64]
    L.sdl_stage_times.argtypes = [vp, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_float), i64]
    L.sdl_last_error.restype = ctypes.c_char_p
    L.sdl_last_error.argtypes = []
    L.sdl_abi_version.restype = i64
    L.sdl_tokenizer_info_get.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(TokenizerInfo)]
    L.sdl_tokenizer_info_get.restype = i64
    for name in ("sdl_batcher_create", "sdl_batcher_push", "sdl_batcher_push_many", "sdl_batcher_next",
                 "sdl_batcher_flush", "sdl_process_device", "sdl_process_device_labels", "sdl_json_text_device",
                 "sdl_pickle_frames_device", "sdl_device_to_host", "sdl_set_profiling",
                 "sdl_stage_times"):
        getattr(L, name).restype = i64
    _lib = L
    return L


def build_id():
    """Content hash of the sources the loaded library was built from (build.source_hash)."""
    return load().sdl_build_id().decode()


def check(rc):
    if rc < 0:
        raise SDLError(rc, load().sdl_last_error().decode(errors="replace"))
    return rc


def tokenizer_info(path, data_dir=DATA_DIR):
    """sdl_tokenizer_info_get: host-side load + checks of a tokenizer (no GPU)."""
    info = TokenizerInfo()
    check(load().sdl_tokenizer_info_get(path.encode(), data_dir.encode(), ctypes.byref(info)))
    return info


def default_config(task):
    c = Config()
    load().sdl_config_default(ctypes.byref(c), task)
    return c


def shard_records(offsets, n_shards):
    """sdl_shard_records (host only): record bounds (numpy u64 [n_shards + 1]) cutting the
    stream described by `offsets` (u64 [n + 1]) into byte-balanced contiguous ranges."""
    import numpy as np
    off = np.ascontiguousarray(offsets, np.uint64)
    bounds = np.zeros(int(n_shards) + 1, np.uint64)
    check(load().sdl_shard_records(off.ctypes.data, len(off) - 1, int(n_shards), bounds.ctypes.data))
    return bounds


def gzip_split_members(buf):
    """sdl_gzip_split_members (host only): member offsets (numpy u64 [n + 1]) of one gzip file."""
    import numpy as np
    L = load()
    b = bytes(buf)
    n = ctypes.c_uint64(0)
    rc = L.sdl_gzip_split_members(b, len(b), None, 0, ctypes.byref(n))
    if rc < 0 and rc != -7:
        check(rc)
    off = np.zeros(n.value + 1, dtype=np.uint64)
    check(L.sdl_gzip_split_members(b, len(b), off.ctypes.data, off.size, ctypes.byref(n)))
    return off


def d2h(handle, dst_numpy, src_ptr, nbytes, stream=None):
    """Device -> host copy into a numpy array through sdl_device_to_host."""
    if nbytes:
        check(load().sdl_device_to_host(handle, dst_numpy.ctypes.data, ctypes.c_void_p(src_ptr), nbytes,
                                        ctypes.c_void_p(stream or None)))
    return dst_numpy
