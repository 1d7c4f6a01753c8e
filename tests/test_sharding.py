"""The N>1 path of bench.py on the CPU (gloo, world_size 2): each rank owns a
contiguous byte-balanced shard of one record stream (the product's
sdl_shard_records; first_record = the global index of its first record), there
is no data-path collective, and the harness only barriers and max-reduces the time.  Because mask keys depend on
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


def shard_rows(rank, nbytes=48 << 10, S=128, B=8, world=2):
    """What rank `rank` of bench.py computes, on the oracle: its arena, its
    global record indices, every row it yields."""
    import sys
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import bench
    import oracle_lib
    # bench.shard is the rank logic bench.py runs: this rank's arena and record indices
    _, arena, offs, order, first = bench.shard(rank, nbytes, world=world)
    texts = [bytes(arena[int(offs[i]):int(offs[i + 1])]) for i in range(len(order))]
    rows = oracle_lib.oracle_rows(oracle_lib.Tok(), texts, S, int(np.float32(S) * np.float32(0.15)), seed=1234, B=B,
                                  first_record=first)
    return texts, first, rows


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    import bench
    texts, first, rows = shard_rows(rank)
    # the harness: barrier, per-rank time, bench's max over ranks
    dist.barrier()
    t = torch.tensor([bench.max_over_ranks(1.0 + rank, world)], dtype=torch.float64)
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
    assert f0 == 0 and f1 == n0  # contiguous ranges of one stream
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


def test_bench_gpus_flag_launches_ranks():
    """`bench.py --gpus 2` without a launcher starts 2 ranks itself (RANK /
    WORLD_SIZE / MASTER_* set per child, no GPU touched in the parent): the
    dry run exercises the same launcher, gloo barrier and max reduction, and
    rank 0's line reports n_gpus == 2 with disjoint shards."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--dry-run", "--gpus", "2", "--steps", "2",
                        "--arena-mib", "2"], capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # only rank 0 prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    r0, r1 = d["ranks"]
    assert (r0["first_record"], r1["first_record"]) == (0, r0["records"])  # one stream, cut in two
    assert r0["checksum"] != r1["checksum"]  # different records
    assert abs(r0["bytes"] - r1["bytes"]) < 20_000  # byte-balanced (within a record)
    total = r0["bytes"] + r1["bytes"]
    assert abs(d["value"] - d["config"]["arena_bytes_per_gpu"] * 2 / d["ms_per_step"] / 1e3) / d["value"] < 0.01
    assert total > 0


def test_bench_gpus_disagreeing_with_world_size_fails():
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--dry-run", "--gpus", "1"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 2 and "WORLD_SIZE" in p.stderr
