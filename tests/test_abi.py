"""The C-ABI library builds for gfx950, loads, and exports every symbol the
header declares; config defaults mirror the reference's masking cases.  No
compute calls here (no GPU in the build container)."""
import ctypes
import os
import re

import pytest

from streaming_data_loader_amd import native

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(REPO, "include", "sdl_batcher.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sdl_[a-z_0-9]+)\s*\(", src)))


def test_header_and_exports_agree(native_lib):
    decl = header_functions()
    assert sorted(native.EXPORTS) == decl
    for name in decl:
        assert hasattr(native_lib, name), name


def test_abi_version(native_lib):
    assert native_lib.sdl_abi_version() == 9


def test_config_defaults_mirror_masking_cases(native_lib):
    c = native.default_config(native.SDL_TASK_MLM)
    assert (c.batch_size, c.sequence_length, c.chunk, c.min_ids) == (4096, 128, 1, 64)  # masking_cases.rs:43
    assert c.mask_length == 19 and c.mask_id == 103  # (128 as f32 * 0.15) as usize; mask 103
    assert (c.avg_span_gap, c.avg_span_size) == (16.0, 2.0)
    m = native.default_config(native.SDL_TASK_MULTI_LABEL)
    assert (m.chunk, m.min_ids, m.number_labels) == (0, 0, 9)


def test_struct_layouts():
    assert ctypes.sizeof(native.Config) == 96  # 8 x i32, 2 x f64, 2 x u64, i32 + 7 reserved
    assert ctypes.sizeof(native.Batch) == 4 * 4 + 8 * 6
    assert ctypes.sizeof(native.DeviceRows) == 8 * 8 + 8 + 8 + 8 + 8
    assert ctypes.sizeof(native.TokenizerInfo) == 6 * 4 + 8 + 6 * 4


def test_struct_layouts_match_header(tmp_path):
    """The ctypes mirrors agree with what a C compiler makes of include/sdl_batcher.h."""
    import shutil
    import subprocess
    cc = shutil.which("gcc") or shutil.which("cc")
    if not cc:
        pytest.skip("no C compiler")
    src = tmp_path / "layout.c"
    src.write_text("""#include <stdio.h>
#include <stddef.h>
#include "sdl_batcher.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(sdl_config), sizeof(sdl_batch), sizeof(sdl_device_rows),
         offsetof(sdl_config, seed), offsetof(sdl_batch, labels_f32), offsetof(sdl_device_rows, d_label_errors),
         offsetof(sdl_device_rows, d_tokenize_errors), sizeof(sdl_tokenizer_info));
  return 0;
}
""")
    exe = tmp_path / "layout"
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    subprocess.run([cc, "-I", inc, str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got == [ctypes.sizeof(native.Config), ctypes.sizeof(native.Batch), ctypes.sizeof(native.DeviceRows),
                   native.Config.seed.offset, native.Batch.labels_f32.offset, native.DeviceRows.d_label_errors.offset,
                   native.DeviceRows.d_tokenize_errors.offset, ctypes.sizeof(native.TokenizerInfo)]


def test_create_without_gpu_fails_loudly(native_lib):
    """The product path never falls back to the CPU."""
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    c = native.default_config(native.SDL_TASK_MLM)
    h = ctypes.c_void_p()
    rc = native_lib.sdl_batcher_create(ctypes.byref(c), native.BERT_PROXY_TOKENIZER.encode(),
                                       native.DATA_DIR.encode(), ctypes.byref(h))
    assert rc == -5 and not h.value
    assert b"no HIP device" in native_lib.sdl_last_error()


def test_kernels_are_gfx950_code_objects(native_lib):
    data = open(native.LIB_PATH, "rb").read()
    assert b"gfx950" in data


@pytest.mark.parametrize("path,kind", [(native.BERT_PROXY_TOKENIZER, 0), (native.GPT2_PROXY_TOKENIZER, 1),
                                       (native.T5_PROXY_TOKENIZER, 2)])
def test_tokenizer_info_host_only(native_lib, path, kind):
    """The host loader accepts the three tokenizer layouts without a GPU."""
    info = native.tokenizer_info(path)
    assert info.kind == kind
    if kind == 2:
        assert info.vocab_size == 32100 and info.unk_id == 2 and info.eos_id == 1 and info.n_added == 103
        assert info.word_table_entries > 32100


def test_tokenizer_info_rejects_unsupported(native_lib, tmp_path):
    import json
    with open(native.T5_PROXY_TOKENIZER, encoding="utf-8") as f:
        tj = json.load(f)
    tj["pre_tokenizer"] = {"type": "Metaspace", "replacement": "\u2581", "add_prefix_space": True}
    p = tmp_path / "t.json"
    p.write_text(json.dumps(tj))
    with pytest.raises(native.SDLError, match="WhitespaceSplit"):
        native.tokenizer_info(str(p))
