#!/usr/bin/env python3
"""Diagnostic: phase cycle split of the WordPiece/BPE chunk kernels (run with
SDL_LIB=var/stamps/libsdl_batcher.so): one process_device over the bench arena."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from streaming_data_loader_amd import native  # noqa: E402
from streaming_data_loader_amd.device import DeviceBatcher  # noqa: E402

task = sys.argv[1] if len(sys.argv) > 1 else "mlm"
mib = int(sys.argv[2]) if len(sys.argv) > 2 else 64
corpus = sys.argv[3] if len(sys.argv) > 3 else "fixture"
t = bench.TASKS[task]
arena, offs, order = bench.build_arena(bench.corpus_records(corpus), mib << 20, seed=0x5D1B)
N, R = len(arena) - 16, len(order)
text = torch.from_numpy(arena).cuda()
off = torch.from_numpy(offs.astype(np.int64)).cuda()
kind = {"mlm": native.SDL_TASK_MLM, "clm": native.SDL_TASK_CLM, "multi-label": native.SDL_TASK_MULTI_LABEL, "span": native.SDL_TASK_SPAN}[task]
tok = {"gpt2": native.GPT2_PROXY_TOKENIZER, "t5": native.T5_PROXY_TOKENIZER}.get(t["tok"], native.BERT_PROXY_TOKENIZER)
db = DeviceBatcher(task=kind, batch_size=t["B"], sequence_length=t["S"], seed=1234, tokenizer=tok)
db.set_profiling(True)
db.process(text.data_ptr(), N, off.data_ptr(), R)
torch.cuda.synchronize()
print(db.stage_times(), file=sys.stderr)
db.close()
