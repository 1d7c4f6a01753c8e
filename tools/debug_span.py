"""Diagnostic: span rows on the device vs the oracle, the first mismatching rows printed
with their positions (run on a GPU box with SDL_SPAN_TWO_PHASE=1 to debug the two-phase path).

    python tools/debug_span.py [S] [B] [gap] [size] [rng_mode]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    import torch
    import oracle_lib
    from streaming_data_loader_amd import native
    from streaming_data_loader_amd.device import DeviceBatcher
    S, B_ = int(sys.argv[1]), int(sys.argv[2])
    gap, size, rm = float(sys.argv[3]), float(sys.argv[4]), int(sys.argv[5])
    with open(os.path.join(REPO, "tests", "golden", "test_records.jsonl"), encoding="utf-8") as f:
        records = [json.loads(x)["text"] for x in f]
    blobs = [r.encode() for r in records]
    db = DeviceBatcher(task=native.SDL_TASK_SPAN, batch_size=B_, sequence_length=S, seed=77,
                       tokenizer=native.T5_PROXY_TOKENIZER, avg_span_gap=gap, avg_span_size=size, rng_mode=rm)
    offs = np.zeros(len(blobs) + 1, np.uint64)
    np.cumsum([len(b) for b in blobs], out=offs[1:])
    arena = np.zeros(int(offs[-1]) + 16, np.uint8)
    arena[:int(offs[-1])] = np.frombuffer(b"".join(blobs), np.uint8)
    ta = torch.from_numpy(arena).cuda()
    to = torch.from_numpy(offs.astype(np.int64)).cuda()
    res = db.process(ta.data_ptr(), int(offs[-1]), to.data_ptr(), len(blobs), 0)
    torch.cuda.synchronize()
    G = res.rows()
    ids, am, tt, lab = res.planes(G + (-G) % B_)
    ob = oracle_lib.OracleBatcherEx(oracle_lib.Encoder("t5", oracle_lib.T5Tok()), oracle_lib.SPAN, B_, S, seed=77,
                                    avg_span_gap=gap, avg_span_size=size, rng_mode=rm)
    want = [r for r in (ob.push(b) for b in blobs) if r is not None]
    while True:
        r = ob.flush()
        if r is None:
            break
        want.append(r)
    cat = {k: np.concatenate([w[k][:w["rows"]] for w in want]) for k in ("input_ids", "labels")}
    shown = 0
    for g in range(G):
        for name, got, exp in (("ids", ids[g], cat["input_ids"][g]), ("labels", lab[g], cat["labels"][g])):
            bad = np.nonzero(got != exp)[0]
            if len(bad) and shown < 6:
                shown += 1
                nz = int(np.count_nonzero(exp)) if name == "ids" else int(np.count_nonzero(exp != -100))
                print(f"row {g} {name}: {len(bad)} bad at {bad[:12].tolist()} (filled {nz})")
                lo = max(int(bad[0]) - 3, 0)
                print("   got ", got[lo:lo + 12].tolist())
                print("   want", exp[lo:lo + 12].tolist())
    print("rows", G, "label errors", res.label_errors(), "oracle", ob.span_errors())


if __name__ == "__main__":
    main()
