#!/usr/bin/env python3
"""Diagnostic builds of libsdl_batcher.so with extra -D macros, for A/B timing
on the GPU (tools/gpu_ab.sh): python tools/build_variants.py NAME=MACRO[,MACRO] ...
Libraries go to var/NAME/ (git-ignored, but they travel to the GPU box; the
objects stay in build/, which does not).

The compile-time switches the sources honour are exactly DIAG_MACROS (every
tuning constant is a constexpr; measured-negative alternates were deleted):
a macro outside this list is refused rather than silently ignored."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from streaming_data_loader_amd import build  # noqa: E402

DIAG_MACROS = {
    # per-phase s_memtime stamps in the tokenizer / inflate kernels, printed at handle
    # destruction (tools/uni_stamps.py, tools/wp_stamps.py, tools/gpu_gz_stamps.sh)
    "SDL_STAMPS": "phase stamps",
    # WordPiece: stage the window and record bits, tokenize nothing (every record 0 ids):
    # the load-only HBM calibration of tools/pmc_calibration.py (var/abl3)
    "SDL_ABLATE": "load-only WordPiece chunk kernel",
    # inflate output batch bytes (tests/test_inflate_fuzz.py builds 256 with the next one)
    "SDL_GZ_OBUF": "inflate output batch bytes",
    "SDL_GZ_ALLOW_SMALL_OBUF": "lift the OBUF >= 512 static_assert (the no-progress exit test)",
}


def check(macros):
    for m in macros:
        name = m.partition("=")[0]
        if name not in DIAG_MACROS:
            raise SystemExit(f"unknown diagnostic macro {name!r}; known: {', '.join(sorted(DIAG_MACROS))}")
    return macros


if __name__ == "__main__":
    for spec in sys.argv[1:]:
        name, _, macros = spec.partition("=")
        defines = check(tuple(m for m in macros.split(",") if m))
        lib = build.build(defines=defines,
                          lib=os.path.join(REPO, "var", name, "libsdl_batcher.so"),
                          build_dir=os.path.join(REPO, "build", "var", name, "obj"))
        print(lib)
