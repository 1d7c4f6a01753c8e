#!/usr/bin/env python3
"""Diagnostic builds of libsdl_batcher.so with extra -D macros, for A/B timing
on the GPU (tools/variants.sh): python tools/build_variants.py NAME=MACRO[,MACRO] ..."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from streaming_data_loader_amd import build  # noqa: E402

for spec in sys.argv[1:]:
    name, _, macros = spec.partition("=")
    d = os.path.join(REPO, "build", "var", name)
    lib = build.build(defines=tuple(m for m in macros.split(",") if m), lib=os.path.join(d, "libsdl_batcher.so"),
                      build_dir=os.path.join(d, "obj"))
    print(lib)
