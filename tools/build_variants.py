#!/usr/bin/env python3
"""Diagnostic builds of libsdl_batcher.so with extra -D macros, for A/B timing
on the GPU (tools/gpu_ab.sh): python tools/build_variants.py NAME=MACRO[,MACRO] ...
Libraries go to var/NAME/ (git-ignored, but they travel to the GPU box; the
objects stay in build/, which does not)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from streaming_data_loader_amd import build  # noqa: E402

for spec in sys.argv[1:]:
    name, _, macros = spec.partition("=")
    lib = build.build(defines=tuple(m for m in macros.split(",") if m),
                      lib=os.path.join(REPO, "var", name, "libsdl_batcher.so"),
                      build_dir=os.path.join(REPO, "build", "var", name, "obj"))
    print(lib)
