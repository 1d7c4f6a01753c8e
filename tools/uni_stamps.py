#!/usr/bin/env python3
"""Diagnostic: phase cycle split of k_unigram_chunks and the long-item counters
(run with SDL_LIB=var/stamps/libsdl_batcher.so)."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from streaming_data_loader_amd import native  # noqa: E402
from streaming_data_loader_amd.device import DeviceBatcher  # noqa: E402

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 64
corpus = sys.argv[2] if len(sys.argv) > 2 else "fixture"
arena, offs, order = bench.build_arena(bench.corpus_records(corpus), mib << 20, seed=0x5D1B)
N, R = len(arena) - 16, len(order)
text = torch.from_numpy(arena).cuda()
off = torch.from_numpy(offs.astype(np.int64)).cuda()
db = DeviceBatcher(task=native.SDL_TASK_SPAN, batch_size=256, sequence_length=512, seed=1234,
                   tokenizer=native.T5_PROXY_TOKENIZER)
db.set_profiling(True)
res = db.process(text.data_ptr(), N, off.data_ptr(), R)
torch.cuda.synchronize()
print(db.stage_times(), "tokenize errors", res.tokenize_errors(), file=sys.stderr)
db.close()
