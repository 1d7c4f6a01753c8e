#!/usr/bin/env python3
"""Device-resident tokenize+mask throughput of the MI355X Batcher.

BASELINE.json metric: "device-resident tokenize+mask MB/s of input text,
seq_len=512, 1/2/4/8 MI355X", quoted on configs[1]: task=mlm (BERT WordPiece,
15% mask), seq_len=512, batch=256.

One step = one pass of the hot path (sdl_process_device) over this rank's text
arena already resident in HBM: tokenize every record, frame, filter, chunk
into rows of 512, mask, and write the packed [rows, 512] int32 planes
(input_ids, attention_mask, token_type_ids, labels) -- every batch of 256
rows the arena yields.  Records are independent, so each rank owns a disjoint
shard of the global record stream (weak scaling, no data-path collective);
the barrier and the max-over-ranks time reduction are the harness's only
communication.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

METRIC = "device-resident tokenize+mask MB/s of input text, seq_len=512, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


_T0 = time.perf_counter()


def log(msg):
    print(f"[bench {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def fixture_records():
    with open(os.path.join(REPO, "tests", "golden", "test_records.jsonl"), encoding="utf-8") as f:
        return [json.loads(l)["text"] for l in f]


def build_arena(records, nbytes, seed):
    """Fixture records (data/test.json.gz) tiled in seeded permutations."""
    blobs = [r.encode("utf-8") for r in records]
    rng = np.random.default_rng(seed)
    order, total = [], 0
    while total < nbytes:
        for i in rng.permutation(len(blobs)):
            order.append(int(i))
            total += len(blobs[i])
            if total >= nbytes:
                break
    offs = np.zeros(len(order) + 1, np.uint64)
    np.cumsum(np.array([len(blobs[i]) for i in order], np.uint64), out=offs[1:])
    arena = np.concatenate([np.frombuffer(blobs[i], np.uint8) for i in order] + [np.zeros(16, np.uint8)])
    return arena, offs, order


def _oracle_stream(ob, blobs, order, start, seconds):
    """Push records order[start], order[start+1], ... (cycling) into one oracle
    Batcher until `seconds` have passed; returns (bytes, records, seconds)."""
    done = n = 0
    i = start
    t0 = time.perf_counter()
    while True:
        b = blobs[order[i % len(order)]]
        ob.push_into(b)
        done += len(b)
        n += 1
        i += 1
        if (n & 63) == 0 and time.perf_counter() - t0 > seconds:
            break
    return done, n, time.perf_counter() - t0


def cpu_baseline(records, order, seconds=12.0, mt_seconds=6.0):
    """The CPU oracle (oracle/sdl_oracle.c, the C restatement of the reference
    Batcher) on a bounded, time-limited sample of the same record stream and
    config: (i) one thread -- the reference runs a single Batcher task -- as
    `value`; (ii) one Batcher per host core on disjoint slices.
    ctypes drops the GIL inside the C calls.  Test-infrastructure code, timed
    only here."""
    import threading
    import oracle_lib
    tok = oracle_lib.Tok()
    blobs = [r.encode("utf-8") for r in records]
    ob = oracle_lib.OracleBatcher(tok, 256, 512, 76, 103, seed=1234)
    done, n, dt = _oracle_stream(ob, blobs, order, 0, seconds)
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    threads = max(1, min(16, ncpu))  # the GPU box grants 16 cores per GPU
    res = [None] * threads
    obs = [oracle_lib.OracleBatcher(tok, 256, 512, 76, 103, seed=1234) for _ in range(threads)]

    def work(t):
        res[t] = _oracle_stream(obs[t], blobs, order, t * (len(order) // threads), mt_seconds)

    th = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    mt_dt = time.perf_counter() - t0
    mt_bytes = sum(r[0] for r in res)
    return {"value": round(done / dt / 1e6, 3), "unit": "MB/s", "cores": 1, "kind": "port",
            "sample": f"{n} records ({done / 1e6:.1f} MB) of rank 0's arena stream (cycled), mlm S=512 B=256, "
                      f"oracle/sdl_oracle.c single-threaded, {dt:.1f} s",
            "all_cores": {"value": round(mt_bytes / mt_dt / 1e6, 3), "unit": "MB/s", "cores": threads,
                          "sample": f"{threads} independent oracle Batchers on disjoint slices, "
                                    f"{mt_bytes / 1e6:.1f} MB in {mt_dt:.1f} s"}}


def load_traffic():
    """HBM bytes per tokenize launch from the committed rocprofv3 PMC summary
    (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, MI355X_MICROARCH.md §HBM)."""
    p = os.path.join(REPO, "profiles", "pmc_wordpiece.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--arena-mib", type=int, default=256)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e", action="store_true", help="also time pinned H2D + kernels + D2H")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from streaming_data_loader_amd import build
    from streaming_data_loader_amd.device import DeviceBatcher

    if not os.path.exists(build.LIB):
        build.build()
    records = fixture_records()
    arena, offs, order = build_arena(records, args.arena_mib << 20, seed=0x5D1B + rank)
    N, R = len(arena) - 16, len(order)
    log(f"rank {rank}: arena {N} bytes, {R} records")
    text = torch.from_numpy(arena).to(dev)
    offsets = torch.from_numpy(offs.astype(np.int64)).to(dev)
    stream = torch.cuda.Stream(device=dev)
    db = DeviceBatcher(batch_size=256, sequence_length=512, seed=1234, device=local)
    first_record = rank * 10_000_000  # disjoint global record indices per shard

    def step():
        return db.process(text.data_ptr(), N, offsets.data_ptr(), R, first_record, stream.cuda_stream)

    for i in range(args.warmup):
        res = step()
        torch.cuda.synchronize(dev)
        log(f"warmup {i} done")
    db.set_profiling(True)
    stage_sum = {}

    def barrier():
        if world > 1:
            dist.barrier()

    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
        # stage times of this step (events on the stream the kernels run on)
        for k, v in db.stage_times().items():
            stage_sum[k] = stage_sum.get(k, 0.0) + v
    torch.cuda.synchronize(dev)
    barrier()
    dt = time.perf_counter() - t0
    log(f"timed {args.steps} steps in {dt:.3f} s")
    db.set_profiling(False)
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    rows, toks = res.rows(), res.tokens()
    stage_ms = {k: v / args.steps for k, v in stage_sum.items()}
    tok_ms = stage_ms["wordpiece_chunks"]
    step_ms = dt / args.steps * 1e3
    total_bytes = N * world * args.steps
    value = total_bytes / dt / 1e6
    # algorithmic bytes of one wordpiece_chunks launch: read the text + record
    # offsets, write the ids (4 B each)
    tok_bytes = N + 8 * (R + 1) + 4 * toks
    achieved = tok_bytes / (tok_ms * 1e-3) / 1e9
    # whole path, per step: text + offsets + the four int32 [rows, 512] planes
    path_bytes = N + 8 * (R + 1) + 16 * rows * 512
    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "MB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(step_ms, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8->int32", "data": "synthetic: data/test.json.gz records tiled (seeded)",
        "config": {"workload": "mlm seq_len=512 batch=256 (BASELINE configs[1]), one step = one rank's "
                               f"{args.arena_mib} MiB text arena -> all packed batches",
                   "task": "mlm", "seq_len": 512, "batch": 256, "arena_bytes_per_gpu": N, "records_per_gpu": R,
                   "rows_per_gpu": rows, "batches_per_gpu": -(-rows // 256), "ids_per_gpu": toks,
                   "tokenizer": "bert-base-uncased layout, offline proxy vocab (30,522)",
                   "parallelism": f"record shards x{world}, no collective"},
        "roofline": {"bound": "hbm", "kernel": "k_wordpiece_chunks", "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5),
                     "traffic": load_traffic(), "algorithmic_bytes_per_launch": tok_bytes,
                     "avg_launch_ms": round(tok_ms, 4)},
        "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
        "path_GBps": round(path_bytes / (step_ms * 1e-3) / 1e9, 2),
    }
    log(f"stages {stage_ms}")
    if args.e2e and rank == 0:
        line["end_to_end"] = end_to_end(records, order)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("cpu baseline ...")
        line["cpu_baseline"] = cpu_baseline(records, order)
    elif rank == 0:
        line["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def end_to_end(records, order, nbytes=64 << 20, reps=2):
    """End-to-end rate of the drop-in host path: records in host memory ->
    sdl_batcher_push_many (pinned staging, H2D, all kernels, D2H of every row,
    GenTokenizer's batch queue on the host) -> finished DataSet batches."""
    from streaming_data_loader_amd import batcher as B
    gt = B.GenTokenizer(B.ModelType.Bert, B.BatchConfig(256, 512), B.Mask(76, 103), B.TokenizerConfig(), seed=1234)
    texts, done = [], 0
    for i in order:
        texts.append(records[i])
        done += len(records[i].encode("utf-8"))
        if done >= nbytes:
            break
    blobs = [t.encode("utf-8") for t in texts]
    gt.create_sync_batches(blobs)  # warm: workspace + pinned staging
    best = None
    for r in range(reps):
        t0 = time.perf_counter()
        out = gt.create_sync_batches(blobs)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
        log(f"e2e rep {r}: {len(out)} batches in {dt:.3f} s")
    return {"MBps": round(done / best / 1e6, 2), "ms": round(best * 1e3, 2), "bytes": done,
            "path": "host records -> sdl_batcher_push_many: pinned H2D, kernels, D2H of all rows, host batch queue"}


if __name__ == "__main__":
    main()
