"""Every SDL_* switch the native sources read is either part of the C ABI
(include/sdl_batcher.h), a diagnostic macro tools/build_variants.py knows,
or an environment hook a test or tool sets -- no orphaned A/B variants."""
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# environment hooks read by the library, and who sets them
ENV_HOOKS = {
    "SDL_SPAN_TWO_PHASE": "tests/test_gpu_span.py",
    "SDL_RAND_SPEC_RHO_PCT": "tests/test_gpu_rand_mode.py",
    "SDL_RAND_REC0": "tests/test_gpu_rand_mode.py",
    "SDL_UNI_ITEM_CAP": "tests/test_gpu_push_direct.py",
    "SDL_SEGMENTS": "tests/test_gpu_parity.py",
    "SDL_SEG_MIN_CHUNKS": "tests/test_gpu_parity.py",
    "SDL_HOST_TIMING": "tools/push_latency.py",
    "SDL_GZ_DEBUG": "tools/gz_single.py",
}


def _names(root, exts):
    out = set()
    for d, _, files in os.walk(root):
        for f in files:
            if f.endswith(exts):
                with open(os.path.join(d, f), encoding="utf-8", errors="replace") as fh:
                    out |= set(re.findall(r"\bSDL_[A-Z0-9_]+", fh.read()))
    return out


def test_every_switch_has_an_owner():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bv", os.path.join(REPO, "tools", "build_variants.py"))
    bv = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bv)
    abi = _names(os.path.join(REPO, "include"), (".h",))
    src = _names(os.path.join(REPO, "streaming_data_loader_amd", "csrc"), (".hip", ".hpp", ".cpp", ".h"))
    orphans = sorted(src - abi - set(bv.DIAG_MACROS) - set(ENV_HOOKS))
    assert not orphans, orphans
    for name, user in ENV_HOOKS.items():
        with open(os.path.join(REPO, user), encoding="utf-8") as fh:
            assert name in fh.read(), (name, user)
