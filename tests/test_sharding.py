"""The N>1 path of bench.py on the CPU (gloo, world_size 2): each rank owns a
disjoint shard of the record stream (its own seeded arena, global record
indices first_record = rank * 10^7), there is no data-path collective, and the
harness only barriers and max-reduces the time.  Because mask keys depend on
(seed, global record index, chunk) only, a shard's rows are the rows the whole
stream would give those records: checked here with the CPU oracle (the GPU
kernels are bit-exact to it, tests/test_gpu_*.py)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def shard_rows(rank, nbytes=48 << 10, S=128, B=8):
    """What rank `rank` of bench.py computes, on the oracle: its arena, its
    global record indices, every row it yields."""
    import sys
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import bench
    import oracle_lib
    recs = bench.fixture_records()
    arena, offs, order = bench.build_arena(recs, nbytes, seed=0x5D1B + rank)
    first = rank * 10_000_000
    texts = [bytes(arena[int(offs[i]):int(offs[i + 1])]) for i in range(len(order))]
    rows = oracle_lib.oracle_rows(oracle_lib.Tok(), texts, S, int(np.float32(S) * np.float32(0.15)), seed=1234, B=B,
                                  first_record=first)
    return texts, first, rows


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    texts, first, rows = shard_rows(rank)
    # the harness: barrier, per-rank time, max over ranks
    dist.barrier()
    t = torch.tensor([1.0 + rank], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    meta = [None] * world
    dist.all_gather_object(meta, (first, len(texts), int(rows.shape[1]), int(np.int64(rows.sum()))))
    if rank == 0:
        out.put((float(t.item()), meta))
    dist.destroy_process_group()


def test_two_rank_shards_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    tmax, meta = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == 2.0  # max over ranks
    (f0, n0, g0, s0), (f1, n1, g1, s1) = meta
    assert f1 >= f0 + n0  # disjoint global record indices
    assert g0 > 0 and g1 > 0
    # each shard's rows, recomputed in this process, match what the rank reported
    for r, (f, n, g, sm) in enumerate(meta):
        _, first, rows = shard_rows(r)
        assert (first, rows.shape[1], int(np.int64(rows.sum()))) == (f, g, sm)


def test_shard_rows_are_the_whole_streams_rows():
    """Rows of a record depend only on (seed, its global index, chunk): a shard
    processed alone equals the same records inside a longer stream."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib
    texts1, first1, rows1 = shard_rows(1, nbytes=24 << 10)
    texts0, _, _ = shard_rows(0, nbytes=24 << 10)
    S = 128
    tok = oracle_lib.Tok()
    # one batcher over shard 0 then shard 1, record indices set per record
    ob = oracle_lib.OracleBatcher(tok, 8, S, 19, 103, 1234)
    planes = []
    for i, t in enumerate(texts0 + texts1):
        ob.set_next_record(i if i < len(texts0) else first1 + (i - len(texts0)))
        r = ob.push(t)
        if r is not None:
            planes.append(r[0][:, :r[1]])
    while True:
        r = ob.flush()
        if r is None:
            break
        planes.append(r[0][:, :r[1]])
    whole = np.concatenate(planes, axis=1)
    n1 = rows1.shape[1]
    np.testing.assert_array_equal(whole[:, -n1:], rows1)
