#!/usr/bin/env python3
"""Device-resident tokenize+mask throughput of the MI355X Batcher.

BASELINE.json metric: "device-resident tokenize+mask MB/s of input text,
seq_len=512, 1/2/4/8 MI355X", quoted on configs[1]: task=mlm (BERT WordPiece,
15% mask), seq_len=512, batch=256 -- the default workload here.

One step = one pass of the hot path (sdl_process_device) over this rank's text
arena already resident in HBM: tokenize every record, frame, filter, chunk
into rows, mask/label, and write the packed [rows, S] int32 planes -- every
batch the arena yields.  Records are independent, so each rank owns a disjoint
shard of the global record stream (weak scaling, no data-path collective);
the barrier and the max-over-ranks time reduction are the harness's only
communication.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--task mlm|span|clm|multi-label|single-class]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)
  python bench.py --gpus N ...   (no launcher: starts the N ranks itself, launch_ranks)

--task selects the other BASELINE configs (not the headline line):
  span         configs[2]: t5 Unigram, seq_len=512, batch=256, T5Data span
               corruption with the reference's Span{16.0, 2.0}
  clm          configs[3]: gpt2 byte-level BPE, seq_len=1024, batch=128
  multi-label  configs[4]: bert WordPiece, seq_len=128, batch=2048, Label::Multi
               indices per record (<= 4 of 9, seed 42); --e2e adds the Arrow
               record path with H2D/D2H.
"""
import argparse
import json
import struct
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

METRIC = "device-resident tokenize+mask MB/s of input text, seq_len=512, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec

TASKS = {
    "mlm": {"S": 512, "B": 256, "tok": "bert", "kernel": "k_wordpiece_chunks", "planes": 4,
            "workload": "mlm seq_len=512 batch=256 (BASELINE configs[1])"},
    # (the tokenize stage the HIP events time: for span the chunk kernel, the two Viterbi
    # launches and the long-item stages; for clm the chunk kernel and k_bpe_long -- their PMC
    # counters are summed over the same launches)
    "span": {"S": 512, "B": 256, "tok": "t5", "kernel": "k_unigram_chunks", "planes": 2.25,
             "pmc_kernels": ["k_unigram_chunks", "k_unigram_viterbi", "k_unigram_long", "k_unigram_huge"],
             "workload": "span t5 Unigram seq_len=512 batch=256 (BASELINE configs[2]; reference Span{16.0, 2.0})"},
    "clm": {"S": 1024, "B": 128, "tok": "gpt2", "kernel": "k_bpe_chunks", "planes": 3,
            "pmc_kernels": ["k_bpe_chunks", "k_bpe_long"],
            "workload": "clm gpt2 byte-BPE seq_len=1024 batch=128 (BASELINE configs[3])"},
    "multi-label": {"S": 128, "B": 2048, "tok": "bert", "kernel": "k_wordpiece_chunks", "planes": 3,
                    "workload": "multi-label seq_len=128 batch=2048 (BASELINE configs[4], B from multi_cases.rs:22)"},
    "single-class": {"S": 128, "B": 2048, "tok": "bert", "kernel": "k_wordpiece_chunks", "planes": 3.0078125,
                     "workload": "single-class seq_len=128 batch=2048 (single_cases.rs Imdb; SURVEY 8(f) row 4)"},
}

_T0 = time.perf_counter()


def log(msg):
    print(f"[bench {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def fixture_records():
    with open(os.path.join(REPO, "tests", "golden", "test_records.jsonl"), encoding="utf-8") as f:
        return [json.loads(l)["text"] for l in f]


def corpus_records(corpus="fixture"):
    """fixture: the reference's data/test.json.gz records; heldout: English
    text never used to build or tune any table (tests/golden/heldout_records.jsonl,
    tools/make_heldout.py)."""
    if corpus == "fixture":
        return fixture_records()
    with open(os.path.join(REPO, "tests", "golden", "heldout_records.jsonl"), encoding="utf-8") as f:
        return [json.loads(l)["text"] for l in f]


def build_order(records, nbytes, seed):
    """The record stream: fixture records (data/test.json.gz) tiled in seeded permutations
    until nbytes of text (record indices into `records`)."""
    lens = [len(r.encode("utf-8")) for r in records]
    rng = np.random.default_rng(seed)
    order, total = [], 0
    while total < nbytes:
        for i in rng.permutation(len(records)):
            order.append(int(i))
            total += lens[i]
            if total >= nbytes:
                break
    return order


def arena_of(records, order):
    blobs = [r.encode("utf-8") for r in records]
    offs = np.zeros(len(order) + 1, np.uint64)
    np.cumsum(np.array([len(blobs[i]) for i in order], np.uint64), out=offs[1:])
    arena = np.concatenate([np.frombuffer(blobs[i], np.uint8) for i in order] + [np.zeros(16, np.uint8)])
    return arena, offs


def build_arena(records, nbytes, seed):
    """Fixture records (data/test.json.gz) tiled in seeded permutations."""
    order = build_order(records, nbytes, seed)
    arena, offs = arena_of(records, order)
    return arena, offs, order


def record_labels(n, seed=42):
    """Label::Multi indices: 0-4 distinct labels of 9 per record."""
    rng = np.random.default_rng(seed)
    k = rng.integers(0, 5, size=n)
    offs = np.zeros(n + 1, np.uint64)
    np.cumsum(k, out=offs[1:])
    vals = np.concatenate([rng.choice(9, size=int(x), replace=False) for x in k]).astype(np.uint32) \
        if n else np.zeros(0, np.uint32)
    return vals, offs


def _oracle_batcher(task, oracle_lib):
    t = TASKS[task]
    if t["tok"] == "gpt2":
        enc = oracle_lib.Encoder("gpt2", oracle_lib.Gpt2Tok())
    elif t["tok"] == "t5":
        enc = oracle_lib.Encoder("t5", oracle_lib.T5Tok())
    else:
        enc = oracle_lib.Encoder("bert", oracle_lib.Tok())
    kind = {"mlm": oracle_lib.MLM, "clm": oracle_lib.CLM, "span": oracle_lib.SPAN,
            "multi-label": oracle_lib.MULTI_LABEL, "single-class": oracle_lib.SINGLE_CLASS}[task]
    return lambda: oracle_lib.OracleBatcherEx(enc, kind, t["B"], t["S"], seed=1234)


def _oracle_stream(ob, blobs, order, labels, start, seconds):
    """Push records order[start], order[start+1], ... (cycling) into one oracle
    Batcher until `seconds` have passed; returns (bytes, records, seconds)."""
    done = n = 0
    i = start
    t0 = time.perf_counter()
    while True:
        k = order[i % len(order)]
        b = blobs[k]
        ob.push_raw(b, labels[k] if labels is not None else None)
        done += len(b)
        n += 1
        i += 1
        if (n & 63) == 0 and time.perf_counter() - t0 > seconds:
            break
    return done, n, time.perf_counter() - t0


def cpu_baseline(task, records, order, seconds=12.0, mt_seconds=6.0):
    """The CPU oracle (oracle/, the C restatement of the reference Batcher) on a
    bounded, time-limited sample of the same record stream and config: (i) one
    thread -- the reference runs a single Batcher task -- as `value`; (ii) one
    Batcher per host core on disjoint slices.  ctypes drops the
    GIL inside the C calls.  Test-infrastructure code, timed only here."""
    import threading
    import oracle_lib
    make = _oracle_batcher(task, oracle_lib)
    blobs = [r.encode("utf-8") for r in records]
    labels = None
    if task == "multi-label":
        vals, offs = record_labels(len(blobs))
        labels = [vals[int(offs[i]):int(offs[i + 1])] for i in range(len(blobs))]
    elif task == "single-class":
        labels = [np.array([i & 1], np.uint32) for i in range(len(blobs))]
    done, n, dt = _oracle_stream(make(), blobs, order, labels, 0, seconds)
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    threads = max(1, min(16, ncpu))  # the GPU box grants 16 cores per GPU
    res = [None] * threads
    obs = [make() for _ in range(threads)]

    def work(t):
        res[t] = _oracle_stream(obs[t], blobs, order, labels, t * (len(order) // threads), mt_seconds)

    th = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    mt_dt = time.perf_counter() - t0
    mt_bytes = sum(r[0] for r in res)
    t = TASKS[task]
    return {"value": round(done / dt / 1e6, 3), "unit": "MB/s", "cores": 1, "kind": "port",
            "sample": f"{n} records ({done / 1e6:.1f} MB) of rank 0's arena stream (cycled), {task} "
                      f"S={t['S']} B={t['B']}, oracle/ C restatement single-threaded, {dt:.1f} s",
            "all_cores": {"value": round(mt_bytes / mt_dt / 1e6, 3), "unit": "MB/s", "cores": threads,
                          "sample": f"{threads} independent oracle Batchers on disjoint slices, "
                                    f"{mt_bytes / 1e6:.1f} MB in {mt_dt:.1f} s"}}


def reference_engine_rate(task, records, order, seconds=6.0):
    """The reference's own tokenizer engine -- HF `tokenizers` (Rust core; the
    reference pins crate 0.13.1, tokenizer_holder.rs:19-28), here its Python
    binding -- encoding the same record stream one record at a time on one
    thread with the same tokenizer.json, as the reference Batcher's single task
    does.  Tokenization only (no masking/batching): an upper bound on the
    reference CPU Batcher's rate.  None when the binding is absent."""
    os.environ.setdefault("RAYON_NUM_THREADS", "1")
    try:
        from tokenizers import Tokenizer
    except Exception:
        return None
    from streaming_data_loader_amd import native
    path = {"gpt2": native.GPT2_PROXY_TOKENIZER, "t5": native.T5_PROXY_TOKENIZER}.get(TASKS[task]["tok"],
                                                                                     native.BERT_PROXY_TOKENIZER)
    tok = Tokenizer.from_file(path)
    done = n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        r = records[order[n % len(order)]]
        tok.encode(r, add_special_tokens=True)
        done += len(r.encode("utf-8"))
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(done / dt / 1e6, 3), "unit": "MB/s", "cores": 1, "kind": "reference engine",
            "sample": f"{n} records ({done / 1e6:.1f} MB) of rank 0's arena stream, tokenizers "
                      f"{getattr(__import__('tokenizers'), '__version__', '?')} Tokenizer.encode, one thread, "
                      f"{dt:.1f} s (tokenization only)"}


PMC_DIR = os.path.join(REPO, "profiles", "pmc")
VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 2  # wave64 VALU instr/s: 256 CUs x 4 SIMD32, 2 cycles each, 2.4 GHz
SALU_ISSUE_PEAK = 256 * 2.4e9  # scalar instr/s: one scalar unit per CU issuing one per cycle


def pmc_path(task, arena_mib, corpus="fixture"):
    return os.path.join(PMC_DIR, f"{task}_{arena_mib}mib" + ("" if corpus == "fixture" else f"_{corpus}") + ".json")


def load_pmc(task, arena_mib, kernel, corpus="fixture"):
    """The committed rocprofv3 --pmc summary of `kernel` (tools/pmc.sh +
    tools/pmc_summary.py) for THIS task, arena size and corpus, or (None,
    reason).  Counters of another task, arena or corpus never describe the
    timed launch, so they are not used."""
    p = pmc_path(task, arena_mib, corpus)
    if not os.path.exists(p):
        return None, f"no PMC summary for task={task} arena={arena_mib} MiB corpus={corpus} ({os.path.relpath(p, REPO)})"
    try:
        with open(p) as f:
            d = json.load(f)
        if d.get("task") != task or int(d.get("arena_mib", -1)) != arena_mib or d.get("corpus", "fixture") != corpus:
            return None, (f"{os.path.relpath(p, REPO)} was collected for task={d.get('task')} "
                          f"arena={d.get('arena_mib')} corpus={d.get('corpus', 'fixture')}")
        # (a template instance is named with its arguments: sdl::k_wordpiece_chunks<false>)
        kernels = kernel if isinstance(kernel, (list, tuple)) else [kernel]
        names = [n for n in d["kernels"] for kk in kernels if n == "sdl::" + kk or n.startswith("sdl::" + kk + "<")]
        if not names:
            raise StopIteration(f"no {kernels} in the summary")
        if len(names) == 1:
            k = d["kernels"][names[0]]
        else:  # the tokenize stage's launches together: counters summed per stage launch
            k = {"launches": max(d["kernels"][n]["launches"] for n in names), "counters": {},
                 "kernels_summed": [n.replace("sdl::", "") for n in names]}
            for n in names:
                for c, v in d["kernels"][n]["counters"].items():
                    k["counters"][c] = k["counters"].get(c, 0.0) + v
        k["_file"] = os.path.relpath(p, REPO)
        return k, None
    except Exception as e:  # a malformed summary is reported, not used
        return None, f"{os.path.relpath(p, REPO)}: {e}"


def stream_calibration():
    """What FETCH_SIZE reports for the chunk kernels' text + offsets stream alone, per byte of
    it: the load-only WordPiece build (SDL_ABLATE=3: stage the 1,088-byte windows, tokenize
    nothing) over the fixture 256 MiB arena (tools/gpu_pmc_load.sh, tools/pmc_calibration.py
    -> profiles/pmc/stream_calibration.json).  None if absent."""
    p = os.path.join(REPO, "profiles", "pmc", "stream_calibration.json")
    try:
        with open(p) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def pmc_traffic(pmc, stream_bytes):
    """HBM bytes per launch from FETCH_SIZE / WRITE_SIZE (KiB units), split by source.

    The guide's gfx950 correction (MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the bytes
    of a 16 B/lane streaming read) does not describe these kernels' reads as a whole: the
    load-only build measures FETCH_SIZE = 0.70 x the stream's bytes (the 1 KiB lane loads
    under-reported, the 32-byte halo loads and offsets not), so a uniform x2 states the stream
    at 1.4x its size.  The stream is therefore counted as its own bytes (`stream_bytes`, text +
    offsets, read once), the calibrated share of FETCH_SIZE (ratio x stream_bytes) is taken
    out, and the rest of FETCH_SIZE -- vocabulary / merge-table probes, list reads, scattered
    4-64 B accesses the x2 does not apply to -- is added as reported, with WRITE_SIZE.  The
    split also keeps the uniform-x2 figure as an upper bound."""
    c = pmc["counters"]
    if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
        return pmc.get("hbm_bytes_per_launch"), None
    fetch, write = c["FETCH_SIZE"] * 1024, c["WRITE_SIZE"] * 1024
    cal = stream_calibration()
    ratio = cal["ratio"] if cal else 0.5
    other = max(fetch - ratio * stream_bytes, 0.0)
    traffic = int(stream_bytes + other + write)
    split = {"stream_read": int(stream_bytes), "probe_and_list_read": int(other), "write": int(write),
             "fetch_size_reported": int(fetch), "stream_fetch_ratio": round(ratio, 4),
             "stream_fetch_ratio_from": "load-only build FETCH_SIZE (profiles/pmc/stream_calibration.json)"
             if cal else "guide's 1/2 (no calibration file)",
             "uniform_x2_upper_bound": int(2 * fetch + write),
             "estimate": "the stream ratio is measured on the WordPiece load-only build and applied to every "
                         "chunk kernel (they share the window geometry); `traffic` is an estimate between "
                         "FETCH_SIZE + WRITE_SIZE as reported and uniform_x2_upper_bound"}
    return traffic, split


def pmc_roofline(pmc, launch_ms, alg_bytes, stream_bytes=0):
    """traffic = HBM bytes per launch (pmc_traffic: the text + offsets stream at its own bytes, the
    rest of FETCH_SIZE past its calibrated share, + WRITE_SIZE); issue = VALU and SALU wave-
    instructions per launch over this run's HIP-event launch time against
    their issue peaks (the byte-walking kernels are bound by the scalar unit:
    one per CU, shared by its four SIMDs); `bound` names the busier one.
    A figure that cannot describe the timed launch (issue above its peak) is
    dropped with the reason."""
    traffic, split = pmc_traffic(pmc, stream_bytes)
    pmc["_split"] = split
    c = pmc["counters"]
    valu, salu = c.get("SQ_INSTS_VALU"), c.get("SQ_INSTS_SALU")
    issue, note = None, None
    if valu:
        secs = launch_ms * 1e-3
        vf, sf = valu / secs / VALU_ISSUE_PEAK, (salu or 0) / secs / SALU_ISSUE_PEAK
        if max(vf, sf) > 1.0:
            note = f"PMC instruction counts over this launch time give issue frac {max(vf, sf):.3f} > 1: not this launch"
        else:
            issue = {"bound": "salu_issue" if sf > vf else "valu_issue", "frac": round(max(vf, sf), 4),
                     "valu_wave_instr_per_launch": int(valu), "salu_wave_instr_per_launch": int(salu or 0),
                     "valu_frac": round(vf, 4), "salu_frac": round(sf, 4),
                     "peak_valu_T_per_s": round(VALU_ISSUE_PEAK / 1e12, 4),
                     "peak_salu_T_per_s": round(SALU_ISSUE_PEAK / 1e12, 4),
                     "wait_frac": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4) if c.get("SQ_WAVE_CYCLES") else None,
                     "source": pmc["_file"]}
    if traffic is not None and traffic < 0.9 * alg_bytes:
        note = (note + "; " if note else "") + f"PMC traffic {traffic} B < algorithmic {alg_bytes} B"
    return traffic, issue, note


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--soak-s", type=float, default=4.0,
                    help="after the timed region (never part of it): re-run the step for this long and check "
                         "that every run writes the same planes as the timed one (device checksums); 0: off")
    ap.add_argument("--task", default="mlm", choices=sorted(TASKS))
    ap.add_argument("--arena-mib", type=int, default=256)
    ap.add_argument("--corpus", default="fixture", choices=["fixture", "heldout"],
                    help="fixture: data/test.json.gz records tiled (default); heldout: English text on the image "
                         "the proxy vocabularies were not trained on (tests/golden/heldout_records.jsonl; "
                         "a second kernel-tuning corpus, not an untouched one)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-heldout", action="store_true",
                    help="skip the held-out corpus leg (by default a fixture run also times the same config on "
                         "the held-out corpus and reports it under `heldout`, beside `value`)")
    ap.add_argument("--rng-mode", type=int, default=0, choices=[0, 1],
                    help="0 the Philox contract (default); 1 the reference's own draws on a per-row StdRng: "
                         "rand 0.8.5 shuffle (mlm masks), rand_distr StandardNormal (span gaps / sizes)")
    ap.add_argument("--e2e", action="store_true", help="also time the host record path (H2D + kernels + D2H)")
    ap.add_argument("--json", action="store_true",
                    help="also time the provider's JsonText filter on the device (JSON lines -> text arena)")
    ap.add_argument("--gz", action="store_true",
                    help="also time the provider's gzip inflate on the device (BGZF members of the JSON lines)")
    ap.add_argument("--e2e-frames", action="store_true",
                    help="end to end from host JSON lines to host pickle frames: H2D, JsonText filter, "
                         "tokenize+mask, transport frames, D2H (the provider -> batcher -> transport path)")
    ap.add_argument("--frames", action="store_true",
                    help="also time the Transport step on the device: every batch -> its serde_pickle frame")
    ap.add_argument("--spawn", action="store_true",
                    help="start the ranks as child processes even for --gpus 1 (tests the launcher)")
    ap.add_argument("--dry-run", action="store_true",
                    help="harness check without a GPU: ranks, gloo barrier/max reduction and the JSON line, "
                         "with a CPU checksum of the arena as the 'step' (never a measurement)")
    return ap.parse_args(argv)


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`--gpus N` without a launcher: start N ranks of this script as child
    processes (one per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set), the way
    torch.distributed.run would.  This parent never touches the GPU and never
    re-execs; it forwards the children's output (rank 0 prints the JSON line)
    and exits with the first non-zero child status."""
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:  # poll every rank: one that fails must not leave its peers waiting in a barrier
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in live:
                    q.kill()
        if live:
            time.sleep(0.05)
    return rc


def rank_env():
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(rank, nbytes, corpus="fixture", world=1):
    """This rank's shard of ONE global record stream (world x nbytes of the corpus records
    tiled in seeded permutations): the product's byte-balanced contiguous split
    (sdl_shard_records, host only), its records materialised, first_record = the global
    index of its first record, so mask keys are those of the whole stream."""
    from streaming_data_loader_amd import native
    records = corpus_records(corpus)
    order = build_order(records, world * nbytes, seed=0x5D1B)
    lens = np.array([len(records[i].encode("utf-8")) for i in order], np.uint64)
    goffs = np.zeros(len(order) + 1, np.uint64)
    np.cumsum(lens, out=goffs[1:])
    bounds = native.shard_records(goffs, world)
    r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
    mine = order[r0:r1]
    arena, offs = arena_of(records, mine)
    return records, arena, offs, mine, r0


def max_over_ranks(dt, world, device=None):
    """The harness's only communication besides the barrier: the slowest rank's time."""
    if world == 1:
        return dt
    import torch
    import torch.distributed as dist
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


class _DevView:
    """__cuda_array_interface__ of a device buffer the library owns (int32)"""
    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<i4", "data": (ptr, False), "version": 3}


def plane_checksums(res, rows, task, dev):
    """Device-side sums of the int32 planes of a result (all elements, and the
    odd ones): a cheap fingerprint of what a step wrote."""
    import torch
    out = []
    for ptr, w in ((res.r.input_ids, task["S"]), (res.r.attention_mask, task["S"]),
                   (res.r.token_type_ids, task["S"]), (res.r.labels, res.r.label_width)):
        if not ptr or rows == 0:
            out.append((0, 0))
            continue
        t = torch.as_tensor(_DevView(ptr, rows * w), device=dev)
        out.append((int(t.sum(dtype=torch.int64)), int(t[1::2].sum(dtype=torch.int64))))
    return out


def determinism_soak(step, res, rows, task, dev, seconds):
    """Re-run the step (outside the timed region) for `seconds` and compare each
    run's rows, tokens and plane checksums with the timed run's: the kernels must
    be deterministic (every mask and span draw is keyed by record, not by
    scheduling).  Keeps the device busy long enough for an external sampler to
    see it; exits 4 on any difference."""
    import torch
    want = (rows, res.tokens(), plane_checksums(res, rows, task, dev))
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < seconds:
        r2 = step()
        torch.cuda.synchronize(dev)
        n += 1
        got = (r2.rows(), r2.tokens(), plane_checksums(r2, r2.rows(), task, dev))
        if got != want:
            print(f"bench.py: run {n} after the timed region differs from it: {got} vs {want}", file=sys.stderr)
            sys.exit(4)
    log(f"determinism soak: {n} more runs in {time.perf_counter() - t0:.1f} s, identical planes")
    return {"runs": n, "seconds": round(time.perf_counter() - t0, 2), "identical": True}


def _build_id():
    from streaming_data_loader_amd import build
    return build.embedded_id(os.environ.get("SDL_LIB") or build.LIB)


def base_line(args, world, step_ms, value, task, N, R, rows, toks):
    S, B = task["S"], task["B"]
    return {
        "metric": METRIC, "value": round(value, 2), "unit": "MB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(step_ms, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8->int32",
        "library_build_id": (_build_id() or "")[:16],
        "data": ("synthetic: data/test.json.gz records tiled (seeded)" if args.corpus == "fixture" else
                 "synthetic: held-out English text on the image (not in the proxy vocabularies' training text; "
                 "also used to tune kernels) tiled (seeded)"),
        "config": {"workload": f"{task['workload']}, one step = one rank's {args.arena_mib} MiB text arena -> "
                               "all packed batches",
                   "task": args.task, "seq_len": S, "batch": B, "corpus": args.corpus,
                   "arena_bytes_per_gpu": N, "records_per_gpu": R,
                   "rows_per_gpu": rows, "batches_per_gpu": -(-rows // B), "ids_per_gpu": toks,
                   "tokenizer": {"gpt2": "gpt2 byte-level BPE layout, offline proxy vocab (50,257)",
                                 "t5": "t5-small layout (Precompiled nmt_nfkc + Unigram), offline proxy vocab (32,100)"}
                                .get(task["tok"], "bert-base-uncased layout, offline proxy vocab (30,522)"),
                   "parallelism": f"record shards x{world}, no collective",
                   "rng": ("rng_mode 1: the reference's draws on a per-row StdRng (rand 0.8.5 shuffle for mlm "
                           "masks, rand_distr 0.4.3 StandardNormal for span gaps / sizes)"
                           if getattr(args, "rng_mode", 0) == 1 else "rng_mode 0: the Philox contract (DESIGN.md §3)")},
    }


def dry_run(args, world, rank):
    """--dry-run: the multi-rank harness on the CPU (gloo): shard, barrier,
    timed 'steps' (a numpy checksum of the arena, NOT the product), max over
    ranks, rank 0's JSON line.  Exercises launch_ranks in CPU tests."""
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    records, arena, offs, order, first = shard(rank, args.arena_mib << 20, args.corpus, world)
    N, R = len(arena) - 16, len(order)
    sums = []
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sums.append(int(arena[:N].sum(dtype=np.uint64)))
    if world > 1:
        dist.barrier()
    dt = max_over_ranks(time.perf_counter() - t0, world)
    meta = [None] * world
    if world > 1:
        dist.all_gather_object(meta, (rank, first, R, N, sums[-1]))
    else:
        meta = [(rank, first, R, N, sums[-1])]
    task = TASKS[args.task]
    if rank == 0:
        line = base_line(args, world, dt / args.steps * 1e3, N * world * args.steps / dt / 1e6, task, N, R, 0, 0)
        line["data"] = "DRY RUN: CPU checksum of the arena, no GPU -- not a measurement"
        line["ranks"] = [{"rank": m[0], "first_record": m[1], "records": m[2], "bytes": m[3], "checksum": m[4]}
                         for m in meta]
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def make_step(task_name, db, records, arena, offs, order, first_record, dev, stream):
    """One step of the hot path over a resident arena: sdl_process_device[_labels]
    (the tensors stay alive in the closure)."""
    import torch
    N, R = len(arena) - 16, len(order)
    text = torch.from_numpy(arena).to(dev)
    offsets = torch.from_numpy(offs.astype(np.int64)).to(dev)
    if task_name == "single-class":  # Label::Single: record i's label is i & 1 (imdb: 2 classes)
        t_lab = torch.from_numpy((np.asarray(order, np.int64) & 1).astype(np.int32)).to(dev)
        t_loff = torch.arange(R + 1, dtype=torch.int64, device=dev)
    elif task_name == "multi-label":
        lv, lo = record_labels(len(records))
        per = [lv[int(lo[i]):int(lo[i + 1])] for i in range(len(records))]
        vals = np.concatenate([per[i] for i in order]).astype(np.int32)
        loff = np.zeros(R + 1, np.int64)
        np.cumsum([len(per[i]) for i in order], out=loff[1:])
        t_lab = torch.from_numpy(vals).to(dev)
        t_loff = torch.from_numpy(loff).to(dev)
    else:
        def step():
            return db.process(text.data_ptr(), N, offsets.data_ptr(), R, first_record, stream.cuda_stream)
        return step

    def step():
        return db.process_labels(text.data_ptr(), N, offsets.data_ptr(), R, t_lab.data_ptr(), t_loff.data_ptr(),
                                 first_record, stream.cuda_stream)
    return step


def heldout_leg(args, db, dev, stream, task, world, rank, barrier):
    """The same config on the held-out corpus (text the proxy vocabularies were not
    trained on), timed like the headline (warmup, barrier + synchronize around
    exactly K steps, max over ranks).  Reported beside `value`, never in its place."""
    import torch
    records, arena, offs, order, first = shard(rank, args.arena_mib << 20, "heldout", world)
    N, R = len(arena) - 16, len(order)
    step = make_step(args.task, db, records, arena, offs, order, first, dev, stream)
    for _ in range(args.warmup):
        res = step()
        torch.cuda.synchronize(dev)
    db.set_profiling(True)
    tok_sum = 0.0
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
        tok_sum += db.stage_times().get("tokenize", 0.0)
    torch.cuda.synchronize(dev)
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0, world, dev)
    db.set_profiling(False)
    tok_err, lab_err = res.tokenize_errors(), res.label_errors()
    toks = res.tokens()
    tok_ms = tok_sum / args.steps
    tok_bytes = N + 8 * (R + 1) + 4 * toks
    achieved = tok_bytes / (tok_ms * 1e-3) / 1e9
    out = {"corpus": "heldout (tests/golden/heldout_records.jsonl tiled, seeded)",
           "value": round(N * world * args.steps / dt / 1e6, 2), "unit": "MB/s",
           "ms_per_step": round(dt / args.steps * 1e3, 4), "arena_bytes_per_gpu": N, "records_per_gpu": R,
           "rows_per_gpu": res.rows(), "ids_per_gpu": toks,
           "errors": {"tokenize": tok_err, "label": lab_err},
           "roofline": {"kernel": task["kernel"], "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5),
                        "algorithmic_bytes_per_launch": tok_bytes, "avg_launch_ms": round(tok_ms, 4)}}
    pmc, note = load_pmc(args.task, args.arena_mib, task.get("pmc_kernels", task["kernel"]), "heldout")
    if pmc is not None:
        traffic, issue, note = pmc_roofline(pmc, tok_ms, tok_bytes, stream_bytes=N + 8 * (R + 1))
        out["roofline"]["traffic"] = traffic
        out["roofline"]["issue"] = issue
    if note:
        out["roofline"]["pmc_note"] = note
    log(f"held-out: {out['value']} MB/s, tokenize {tok_ms:.4f} ms")
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus > 1 or args.spawn):
        sys.exit(launch_ranks(args.gpus, [a for a in argv if a != "--spawn"]))
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}: launch one rank per GPU with "
              f"--nproc-per-node equal to --gpus", file=sys.stderr)
        sys.exit(2)
    world, rank, local = rank_env()
    if args.dry_run:
        return dry_run(args, world, rank)
    task = TASKS[args.task]
    S, B = task["S"], task["B"]

    import torch
    import torch.distributed as dist

    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from streaming_data_loader_amd import build, native
    from streaming_data_loader_amd.device import DeviceBatcher

    if not os.path.exists(build.LIB):
        build.build()
    records, arena, offs, order, first_record = shard(rank, args.arena_mib << 20, args.corpus, world)
    N, R = len(arena) - 16, len(order)
    log(f"rank {rank}/{world}: task {args.task}, corpus {args.corpus}, arena {N} bytes, {R} records, "
        f"first record {first_record}")
    stream = torch.cuda.Stream(device=dev)
    kind = {"mlm": native.SDL_TASK_MLM, "clm": native.SDL_TASK_CLM, "span": native.SDL_TASK_SPAN,
            "multi-label": native.SDL_TASK_MULTI_LABEL, "single-class": native.SDL_TASK_SINGLE_CLASS}
    tok_path = {"gpt2": native.GPT2_PROXY_TOKENIZER, "t5": native.T5_PROXY_TOKENIZER}.get(task["tok"],
                                                                                          native.BERT_PROXY_TOKENIZER)
    db = DeviceBatcher(task=kind[args.task], batch_size=B, sequence_length=S, seed=1234, device=local,
                       tokenizer=tok_path, rng_mode=args.rng_mode)
    step = make_step(args.task, db, records, arena, offs, order, first_record, dev, stream)

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
        # stage times of this step (hipEvents on the stream the kernels run on)
        for k, v in db.stage_times().items():
            stage_sum[k] = stage_sum.get(k, 0.0) + v
    torch.cuda.synchronize(dev)
    barrier()
    dt = time.perf_counter() - t0
    log(f"timed {args.steps} steps in {dt:.3f} s")
    db.set_profiling(False)
    dt = max_over_ranks(dt, world, dev)

    # capacity flags: a run that dropped text or clamped labels is not a measurement
    tok_err, lab_err = res.tokenize_errors(), res.label_errors()
    if tok_err or lab_err:
        print(f"bench.py: rank {rank}: tokenize_errors={tok_err:#x} label_errors={lab_err} -- the timed run "
              "dropped or clamped data (include/sdl_batcher.h d_tokenize_errors / d_label_errors)", file=sys.stderr)
        sys.exit(3)

    rows, toks = res.rows(), res.tokens()
    soak = determinism_soak(step, res, rows, task, dev, args.soak_s) if args.soak_s > 0 else None
    stage_ms = {k: v / args.steps for k, v in stage_sum.items()}
    tok_ms = stage_ms["tokenize"]
    step_ms = dt / args.steps * 1e3
    value = N * world * args.steps / dt / 1e6
    # algorithmic bytes of one tokenize launch: read the text + record offsets,
    # write the ids (4 B each)
    tok_bytes = N + 8 * (R + 1) + 4 * toks
    achieved = tok_bytes / (tok_ms * 1e-3) / 1e9
    # whole path, per step: text + offsets + the int32 [rows, S] planes
    path_bytes = N + 8 * (R + 1) + int(4 * task["planes"] * rows * S)
    line = base_line(args, world, step_ms, value, task, N, R, rows, toks)
    pmc, pmc_note = load_pmc(args.task, args.arena_mib, task.get("pmc_kernels", task["kernel"]), args.corpus)
    traffic, issue = None, None
    if pmc is not None:
        traffic, issue, pmc_note = pmc_roofline(pmc, tok_ms, tok_bytes, stream_bytes=N + 8 * (R + 1))
    # achieved / peak / frac are against HBM (the metric's roofline); `bound`
    # names the roofline that binds the kernel: the busier issue unit when the
    # PMC summary shows it closer to its peak than HBM traffic is to its own
    hbm_frac = achieved / HBM_PEAK_GBPS
    # the HBM side of the verdict takes the largest of the algorithmic bytes, the calibrated
    # traffic and the uniform-x2 upper bound, so the calibration cannot tip it toward "issue"
    hbm_frac_hi = hbm_frac
    if traffic is not None:
        hbm_frac_hi = max(hbm_frac_hi, traffic / (tok_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS)
    if pmc is not None and pmc.get("_split"):
        hbm_frac_hi = max(hbm_frac_hi, pmc["_split"]["uniform_x2_upper_bound"] / (tok_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS)
    bound = issue["bound"] if issue is not None and issue["frac"] > hbm_frac_hi else "hbm"
    if soak is not None:
        line["determinism"] = soak
    line["roofline"] = {"bound": bound, "kernel": task["kernel"], "achieved": round(achieved, 2),
                        "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(hbm_frac, 5),
                        "traffic": traffic, "issue": issue,
                        "traffic_split": pmc.get("_split") if pmc is not None else None,
                        "algorithmic_bytes_per_launch": tok_bytes, "avg_launch_ms": round(tok_ms, 4),
                        "hbm_frac_upper": round(hbm_frac_hi, 5)}
    if pmc is not None and pmc.get("kernels_summed"):  # (the stage's launches: counters summed)
        line["roofline"]["kernels"] = pmc["kernels_summed"]
    if bound != "hbm":
        line["roofline"]["bound_note"] = (f"{bound} at {issue['frac']:.2f} of its issue peak binds this kernel; "
                                          "achieved/peak/frac are its algorithmic HBM bytes against 8 TB/s")
    if pmc_note:
        line["roofline"]["pmc_note"] = pmc_note
    line["stage_ms"] = {k: round(v, 4) for k, v in stage_ms.items()}
    line["path_GBps"] = round(path_bytes / (step_ms * 1e-3) / 1e9, 2)
    line["errors"] = {"tokenize": tok_err, "label": lab_err}
    log(f"stages {stage_ms}")
    if args.e2e and rank == 0:
        line["end_to_end"] = end_to_end(args.task, records, order)
    if args.json and rank == 0:
        line["provider_json"] = provider_json(db, records, order, dev, args.steps, args.warmup, step_ms)
    if args.gz and rank == 0:
        line["provider_gzip"] = provider_gzip(db, records, order, dev, args.steps, args.warmup, step_ms,
                                             json_mib=args.arena_mib, N_text=N)
    if args.frames and rank == 0:
        line["transport_frames"] = transport_frames(db, res, args.task, stream, dev, args.steps, args.warmup,
                                                    not args.no_cpu_baseline)
    if args.e2e_frames and rank == 0 and args.task in ("mlm", "clm", "span"):
        # last: it reuses the handle's workspace (the step's planes are overwritten)
        line["end_to_end_frames"] = end_to_end_frames(db, records, order, dev, stream, args.task)
    if args.corpus == "fixture" and not args.no_heldout:  # (after the legs that reuse the step's result)
        line["heldout"] = heldout_leg(args, db, dev, stream, task, world, rank, barrier)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("cpu baseline ...")
        line["cpu_baseline"] = cpu_baseline(args.task, records, order)
        line["cpu_baseline"]["reference_engine"] = reference_engine_rate(args.task, records, order)
    elif rank == 0:
        line["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def transport_frames(db, res, task_name, stream, dev, steps, warmup, with_cpu):
    """Transport step on the device (sdl_pickle_frames_device): every batch of
    this step (full batches + the flushed partial one) -> the serde_pickle
    frame the reference's Transport sends (zmq_transmit.rs:71).  Timed with HIP
    events on the stream the kernels run on.  Algorithmic bytes per launch:
    the int32/f32 plane elements read (4 B) + the frame bytes written."""
    import torch
    rows = res.rows()
    fr = None
    for _ in range(warmup):
        fr = db.pickle_frames(res, rows, True, stream.cuda_stream)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        fr = db.pickle_frames(res, rows, True, stream.cuda_stream)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / steps
    t = TASKS[task_name]
    B, S = t["B"], t["S"]
    nb = len(fr)
    LW = {"span": S // 4, "multi-label": 9, "single-class": 1}.get(task_name, S)
    n_planes = {"mlm": 3, "multi-label": 3, "single-class": 3}.get(task_name, 2)
    rows_full = nb * B
    lab_rows = rows if task_name in ("mlm", "multi-label", "single-class") else rows_full
    elems = n_planes * rows_full * S + lab_rows * LW
    alg = 4 * elems + int(fr.f.total_bytes)
    achieved = alg / (ms * 1e-3) / 1e9
    out = {"frames": nb, "frame_bytes": int(fr.f.frame_bytes), "total_bytes": int(fr.f.total_bytes),
           "ms": round(ms, 4), "frame_MBps": round(fr.f.total_bytes / ms / 1e3, 2),
           "roofline": {"bound": "hbm", "kernel": "k_frame_rows", "achieved": round(achieved, 2),
                        "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5),
                        "algorithmic_bytes_per_launch": alg, "avg_launch_ms": round(ms, 4)}}
    if with_cpu:
        # the C restatement of serde_pickle (single thread) on a bounded sample of the same batches
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_lib
        k = min(nb, 24 if S * B >= 65536 else 96)
        ids, am, tt, lab = res.planes(k * B)
        t0, done, nfr = time.perf_counter(), 0, 0
        while time.perf_counter() - t0 < 5.0:
            for b in range(k):
                sl = slice(b * B, (b + 1) * B)
                done += len(oracle_lib.pickle_dataset(task_name, B, S, LW, B, ids[sl], am[sl],
                                                      None if tt is None else tt[sl], lab[sl]))
                nfr += 1
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(done / dt / 1e6, 2), "unit": "MB/s of frames", "cores": 1,
                               "kind": "port", "sample": f"{nfr} frames ({k} distinct batches of this step), "
                                                         f"oracle/orc_pickle.c single-threaded, {dt:.1f} s"}
    return out


def end_to_end_frames(db, records, order, dev, stream, task_name, nbytes=64 << 20, reps=3):
    """The whole hot path from host memory to host memory, as north_star frames it
    (a JSON-lines stream in, the bytes the Transport socket sends out): JSON lines
    in pinned host memory -> H2D -> sdl_json_text_device (the Provider's JsonText
    filter) -> sdl_process_device (tokenize + mask) -> sdl_pickle_frames_device
    (serde_pickle frames of every batch, the flushed partial one included) -> D2H
    into pinned host memory.  Rate = text bytes / wall time; sequential stages on
    one stream (no copy/compute overlap)."""
    import torch
    lines, done = [], 0
    for i, k in enumerate(order):
        lines.append(json.dumps({"id": i, "text": records[k]}).encode("utf-8"))
        done += len(records[k].encode("utf-8"))
        if done >= nbytes:
            break
    buf = b"\n".join(lines) + b"\n"
    host = torch.zeros(len(buf) + 32, dtype=torch.uint8).pin_memory()
    host[:len(buf)] = torch.frombuffer(bytearray(buf), dtype=torch.uint8)
    d_json = torch.empty(len(buf) + 32, dtype=torch.uint8, device=dev)
    out_host = None
    best, info = None, {}
    for r in range(reps + 1):  # first pass warms the workspaces
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            d_json.copy_(host, non_blocking=True)
        jt = db.json_text(d_json.data_ptr(), len(buf), stream.cuda_stream)
        res = db.process(jt.d_text, jt.text_bytes, jt.d_offsets, jt.n_records, 0, stream.cuda_stream)
        rows = res.rows()
        fr = db.pickle_frames(res, rows, True, stream.cuda_stream)
        total = int(fr.f.total_bytes)
        if out_host is None or out_host.numel() < total:
            out_host = torch.empty(total, dtype=torch.uint8).pin_memory()
        from streaming_data_loader_amd import native
        native.d2h(db._h, out_host.numpy(), fr.f.d_frames, total, stream.cuda_stream)
        dt = time.perf_counter() - t0
        if r:
            best = dt if best is None else min(best, dt)
        info = {"records": int(jt.n_records), "rows": rows, "frames": len(fr), "frame_bytes": total}
    assert info["records"] == len(lines)
    out = {"MBps": round(done / best / 1e6, 2), "ms": round(best * 1e3, 2), "text_bytes": done,
           "json_bytes": len(buf), **info,
           "path": "pinned host JSON lines -> H2D -> JsonText filter -> tokenize+mask -> serde_pickle frames -> "
                   "D2H to pinned host (sequential, one stream)"}
    # the same from the reference's input format: the JSON lines gzip-compressed (BGZF
    # members of 65,280 bytes, zlib level 6) in pinned host memory -> H2D of the compressed
    # bytes and member offsets -> sdl_gzip_inflate_device -> JsonText -> tokenize+mask -> frames -> D2H
    import zlib
    from concurrent.futures import ThreadPoolExecutor
    from streaming_data_loader_amd import native
    parts = [buf[i:i + 65280] for i in range(0, len(buf), 65280)]

    def bgzf_member(p):
        co = zlib.compressobj(6, zlib.DEFLATED, -15)
        c = co.compress(p) + co.flush()
        m = b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00\x00\x00" + c + \
            struct.pack("<II", zlib.crc32(p), len(p))
        return m[:16] + struct.pack("<H", len(m) - 1) + m[18:]
    with ThreadPoolExecutor(16) as ex:
        gz = b"".join(ex.map(bgzf_member, parts))
    moff = native.gzip_split_members(gz)
    gz_host = torch.zeros(len(gz) + 32, dtype=torch.uint8).pin_memory()
    gz_host[:len(gz)] = torch.frombuffer(bytearray(gz), dtype=torch.uint8)
    off_host = torch.from_numpy(moff.view(np.int64).copy()).pin_memory()
    d_gz = torch.empty(len(gz) + 32, dtype=torch.uint8, device=dev)
    d_moff = torch.empty(len(moff), dtype=torch.int64, device=dev)
    best_gz = None
    for r in range(reps + 1):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            d_gz.copy_(gz_host, non_blocking=True)
            d_moff.copy_(off_host, non_blocking=True)
        z = db.gzip_inflate(d_gz.data_ptr(), len(gz), d_moff.data_ptr(), len(moff) - 1, stream.cuda_stream)
        jt = db.json_text(z.d_out, int(z.out_bytes), stream.cuda_stream)
        res = db.process(jt.d_text, jt.text_bytes, jt.d_offsets, jt.n_records, 0, stream.cuda_stream)
        fr = db.pickle_frames(res, res.rows(), True, stream.cuda_stream)
        native.d2h(db._h, out_host.numpy(), fr.f.d_frames, int(fr.f.total_bytes), stream.cuda_stream)
        dt = time.perf_counter() - t0
        if r:
            best_gz = dt if best_gz is None else min(best_gz, dt)
        assert int(z.out_bytes) == len(buf) and int(jt.n_records) == len(lines)
        assert int(fr.f.total_bytes) == info["frame_bytes"]
    out["from_gzip"] = {"MBps": round(done / best_gz / 1e6, 2), "ms": round(best_gz * 1e3, 2), "gz_bytes": len(gz),
                        "members": len(moff) - 1,
                        "path": "pinned host BGZF .json.gz -> H2D -> gzip inflate -> JsonText -> tokenize+mask -> "
                                "serde_pickle frames -> D2H to pinned host (sequential, one stream)"}
    # the same, pipelined in the library (sdl_json_to_frames): chunks cut at line ends,
    # chunk k's frames copied out while chunk k+1 is copied in and computed
    # the link's own rate: the frame bytes alone, device -> pinned host (the bound of this path)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(3):
        native.d2h(db._h, out_host.numpy(), fr.f.d_frames, info["frame_bytes"], stream.cuda_stream)
    d2h_s = (time.perf_counter() - t0) / 3
    out["d2h_only"] = {"GBps": round(info["frame_bytes"] / d2h_s / 1e9, 2), "ms": round(d2h_s * 1e3, 2),
                       "text_MBps_bound": round(done / d2h_s / 1e6, 2),
                       "note": "hipMemcpyAsync of the frames alone: the PCIe D2H bound of this path"}
    pinned_json = host[:len(buf)].numpy()  # the pinned copy the sequential path reads
    for chunk_mib, src, kind in ((8, buf, "pageable"), (8, pinned_json, "pinned"), (12, pinned_json, "pinned"),
                                 (16, pinned_json, "pinned"), (24, pinned_json, "pinned"),
                                 (32, pinned_json, "pinned")):
        best_p, st = None, None
        for r in range(reps + 1):
            _, st = db.json_to_frames(src, chunk_bytes=chunk_mib << 20, collect=False)
            if r:
                best_p = st.seconds if best_p is None else min(best_p, st.seconds)
        assert st.n_records == len(lines) and st.n_frames == info["frames"] and st.frame_bytes == info["frame_bytes"]
        out.setdefault("pipelined", []).append(
            {"MBps": round(done / best_p / 1e6, 2), "ms": round(best_p * 1e3, 2), "chunk_MiB": chunk_mib,
             "input": kind, "chunks": int(st.n_chunks), "frame_GBps_d2h": round(st.frame_bytes / best_p / 1e9, 2),
             "host_ms": {k: round(v * 1e3, 2) for k, v in zip(("json_text", "tokenize_rows", "frames_issue",
                                                                "delivery_wait"), st.host_wait)},
             "path": f"{kind} host JSON lines -> sdl_json_to_frames (H2D | JsonText + tokenize+mask + frames | D2H "
                     "on three streams) -> host frames"})
    return out


def provider_json(db, records, order, dev, steps, warmup, step_ms):
    """SourceFilter::JsonText on the device (sdl_json_text_device): this rank's
    record stream as JSON lines ({"id", "title", "text"}, json.dumps) already in
    HBM -> the text arena + offsets the Batcher consumes.  Reports JSON MB/s and
    the JSON-lines -> batches rate with the step time measured above."""
    import torch
    lines = [json.dumps({"id": i, "title": f"t{i}", "text": records[k]}).encode("utf-8") for i, k in enumerate(order)]
    buf = b"\n".join(lines) + b"\n"
    a = np.zeros(len(buf) + 32, np.uint8)
    a[:len(buf)] = np.frombuffer(buf, np.uint8)
    d = torch.from_numpy(a).to(dev)
    for _ in range(warmup):
        out = db.json_text(d.data_ptr(), len(buf))
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        out = db.json_text(d.data_ptr(), len(buf))
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / steps * 1e3
    text = sum(len(records[k].encode("utf-8")) for k in order)
    return {"json_MBps": round(len(buf) / ms / 1e3, 2), "ms": round(ms, 4), "json_bytes": len(buf),
            "records": int(out.n_records), "text_bytes": int(out.text_bytes), "text_bytes_expected": text,
            "invalid_lines": int(out.n_invalid),
            "json_to_batches_MBps": round(len(buf) / (ms + step_ms) / 1e3, 2),
            "note": "host-timed (the call synchronises twice to size its outputs); JSON bytes / time"}


def provider_gzip(db, records, order, dev, steps, warmup, step_ms, json_mib=64, block=65280, N_text=256 << 20):
    """The provider's gzip inflate on the device (sdl_gzip_inflate_device): this
    rank's record stream as JSON lines (as provider_json), gzip-compressed as
    BGZF members of `block` input bytes (zlib level 6), already in HBM -> the
    inflated JSON lines (CRC-32 and ISIZE checked) -> JsonText -> text arena.
    CPU beside it: zlib inflate of the same lines as ONE gzip member on one
    thread (what the reference's GzipDecoder does), and the BGZF members on 16
    threads."""
    import zlib
    import torch
    from concurrent.futures import ThreadPoolExecutor
    from streaming_data_loader_amd import native
    lines, size = [], 0
    for i, k in enumerate(order):
        ln = json.dumps({"id": i, "title": f"t{i}", "text": records[k]}).encode("utf-8") + b"\n"
        lines.append(ln)
        size += len(ln)
        if size >= json_mib << 20:
            break
    buf = b"".join(lines)
    t0 = time.perf_counter()
    parts = [buf[i:i + block] for i in range(0, len(buf), block)]
    with ThreadPoolExecutor(16) as ex:
        def raw(p):
            co = zlib.compressobj(6, zlib.DEFLATED, -15)
            return co.compress(p) + co.flush()
        comp = list(ex.map(raw, parts))
    members = []
    for p, c in zip(parts, comp):
        hdr = b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00"
        m = hdr + b"\x00\x00" + c + struct.pack("<II", zlib.crc32(p), len(p))
        members.append(m[:16] + struct.pack("<H", len(m) - 1) + m[18:])
    gz = b"".join(members)
    log(f"gzip: {len(buf) / 1e6:.1f} MB JSON -> {len(gz) / 1e6:.1f} MB in {len(members)} BGZF members "
        f"({time.perf_counter() - t0:.1f} s to compress)")
    off = native.gzip_split_members(gz)
    assert len(off) == len(members) + 1
    a = np.zeros(len(gz) + 32, np.uint8)
    a[:len(gz)] = np.frombuffer(gz, np.uint8)
    d_gz = torch.from_numpy(a).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    n = len(members)

    def inflate():
        return db.gzip_inflate(d_gz.data_ptr(), len(gz), d_off.data_ptr(), n)
    for _ in range(warmup):
        out = inflate()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        out = inflate()
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / steps * 1e3
    assert int(out.out_bytes) == len(buf) and int(out.n_bad) == 0
    chk = np.zeros(min(len(buf), 1 << 20), np.uint8)
    native.d2h(db._h, chk, out.d_out, chk.nbytes)
    assert chk.tobytes() == buf[:chk.size], "device inflate differs from the JSON lines"
    t0 = time.perf_counter()
    for _ in range(steps):
        out = inflate()
        jt = db.json_text(out.d_out, int(out.out_bytes))
    torch.cuda.synchronize(dev)
    ms_text = (time.perf_counter() - t0) / steps * 1e3
    # the reference's own input shape: the same lines as ONE gzip member (zlib level 6), which the
    # device inflates in chunks (a header search per chunk, chunks checked against each other)
    co = zlib.compressobj(6, zlib.DEFLATED, 31)
    single = co.compress(buf) + co.flush()
    a1 = np.zeros(len(single) + 32, np.uint8)
    a1[:len(single)] = np.frombuffer(single, np.uint8)
    d_one = torch.from_numpy(a1).to(dev)
    d_off1 = torch.from_numpy(np.array([0, len(single)], np.int64)).to(dev)

    def inflate_one():
        return db.gzip_inflate(d_one.data_ptr(), len(single), d_off1.data_ptr(), 1)
    for _ in range(max(warmup, 1)):
        out1 = inflate_one()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        out1 = inflate_one()
    torch.cuda.synchronize(dev)
    ms1 = (time.perf_counter() - t0) / steps * 1e3
    assert int(out1.out_bytes) == len(buf) and int(out1.n_bad) == 0
    full = np.zeros(len(buf), np.uint8)
    native.d2h(db._h, full, out1.d_out, full.nbytes)
    assert full.tobytes() == buf, "device inflate of the single member differs from the JSON lines"
    del full
    t0 = time.perf_counter()
    for _ in range(steps):
        out1 = inflate_one()
        jt1 = db.json_text(out1.d_out, int(out1.out_bytes))
    torch.cuda.synchronize(dev)
    ms1_text = (time.perf_counter() - t0) / steps * 1e3
    assert int(jt1.n_records) == int(jt.n_records)
    # CPU: one member on one thread (the reference), BGZF members on 16 threads
    t0 = time.perf_counter()
    assert len(zlib.decompress(single, 31)) == len(buf)
    cpu1 = time.perf_counter() - t0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(16) as ex:
        got = sum(ex.map(lambda m: len(zlib.decompress(m, 31)), members))
    cpu16 = time.perf_counter() - t0
    assert got == len(buf)
    return {"inflated_MBps": round(len(buf) / ms / 1e3, 2), "compressed_MBps": round(len(gz) / ms / 1e3, 2),
            "ms": round(ms, 4), "json_bytes": len(buf), "gz_bytes": len(gz), "members": n,
            "gz_to_text_ms": round(ms_text, 4), "gz_to_text_MBps": round(len(buf) / ms_text / 1e3, 2),
            "records": int(jt.n_records),
            "gz_to_batches_MBps": round(len(buf) / (ms_text + step_ms * len(buf) / N_text) / 1e3, 2),
            "single_member": {"inflated_MBps": round(len(buf) / ms1 / 1e3, 2), "ms": round(ms1, 4),
                              "gz_bytes": len(single),
                              "gz_to_text_ms": round(ms1_text, 4),
                              "gz_to_text_MBps": round(len(buf) / ms1_text / 1e3, 2),
                              "gz_to_batches_MBps": round(len(buf) / (ms1_text + step_ms * len(buf) / N_text) / 1e3,
                                                          2),
                              "path": "one gzip member (zlib level 6) in HBM -> sdl_gzip_inflate_device (chunked: "
                                      "header search, chunks in parallel, window chain, CRC-32 + ISIZE), host-timed"},
            "cpu_zlib_1thread_one_member_MBps": round(len(buf) / cpu1 / 1e6, 2),
            "cpu_zlib_16threads_bgzf_MBps": round(len(buf) / cpu16 / 1e6, 2),
            "note": "host-timed, includes the call's two synchronisations (trailer sizes, status); "
                    "MB/s of inflated JSON unless named; gz_to_batches scales the step time to this text"}


def end_to_end(task, records, order, nbytes=64 << 20, reps=2):
    """End-to-end rate of the drop-in host path: records in host memory ->
    sdl_batcher_push_many (pinned staging, H2D, all kernels, D2H of every row,
    the reference's batch cadence on the host) -> finished DataSet batches.
    multi-label: the records arrive as Arrow record batches (sentence: utf8,
    labels: list<int64>) and are fed from the column buffers."""
    from streaming_data_loader_amd import batcher as Bt
    from streaming_data_loader_amd import native
    t = TASKS[task]
    texts, done = [], 0
    for i in order:
        texts.append(records[i])
        done += len(records[i].encode("utf-8"))
        if done >= nbytes:
            break
    if task == "single-class":
        import pyarrow as pa
        table = pa.table({"text": pa.array(texts, pa.utf8()),
                          "label": pa.array([i & 1 for i in order[:len(texts)]], pa.int64())})
        batches = table.to_batches(max_chunksize=65536)
        sb = Bt.SimpleBatcher(Bt.ModelType.Bert, Bt.SingleClass(), Bt.BatchConfig(t["B"], t["S"]),
                              Bt.TokenizerConfig())
        run = lambda: [ds for b in batches for ds in sb.push_arrow(b)]  # noqa: E731
        path = "Arrow record batches (text, label) -> SimpleBatcher.push_arrow (column buffers, pinned H2D, kernels, D2H)"
    elif task == "multi-label":
        import pyarrow as pa
        lv, lo = record_labels(len(records))
        labs = [lv[int(lo[i]):int(lo[i + 1])].astype(np.int64) for i in range(len(records))]
        table = pa.table({"sentence": pa.array(texts, pa.utf8()),
                          "labels": pa.array([labs[i] for i in order[:len(texts)]], pa.list_(pa.int64()))})
        batches = table.to_batches(max_chunksize=65536)
        sb = Bt.SimpleBatcher(Bt.ModelType.Bert, Bt.MultiLabel(9), Bt.BatchConfig(t["B"], t["S"]), Bt.TokenizerConfig())
        run = lambda: [ds for b in batches for ds in sb.push_arrow(b)]  # noqa: E731
        path = "Arrow record batches -> SimpleBatcher.push_arrow (column buffers, pinned H2D, kernels, D2H)"
    else:
        tt = {"mlm": Bt.TaskType.Mlm, "clm": Bt.TaskType.Clm, "span": Bt.TaskType.Span}[task]
        cfg = Bt.get_case(tt, False, t["S"], t["B"], 1234)
        gt = Bt.GenTokenizer.from_config(cfg)
        blobs = [x.encode("utf-8") for x in texts]
        run = lambda: gt.create_sync_batches(blobs)  # noqa: E731
        path = "host records -> sdl_batcher_push_many: pinned H2D, kernels, D2H of all rows, host batch queue"
    out = run()  # warm: workspace, pinned staging and the batch pool
    best = None
    for r in range(reps):
        out = None  # a consumer releases its batches: their pinned blocks are recycled
        t0 = time.perf_counter()
        out = run()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
        log(f"e2e rep {r}: {len(out)} batches in {dt:.3f} s")
    res = {"MBps": round(done / best / 1e6, 2), "ms": round(best * 1e3, 2), "bytes": done, "path": path}
    if task in ("mlm", "clm", "span"):
        # the same records handed over as one host arena + offsets (the form an Arrow utf8
        # column or the JsonText output already has): the C-ABI host path without the
        # Python mirror's per-record join
        arena = np.frombuffer(b"".join(blobs), np.uint8)
        offs = np.zeros(len(blobs) + 1, np.uint64)
        np.cumsum([len(x) for x in blobs], out=offs[1:])
        best_a = None
        for r in range(reps):
            out = None
            t0 = time.perf_counter()
            out = gt.push_arena(arena, offs)
            dt = time.perf_counter() - t0
            best_a = dt if best_a is None else min(best_a, dt)
        res["from_arena"] = {"MBps": round(done / best_a / 1e6, 2), "ms": round(best_a * 1e3, 2),
                             "path": "host arena + offsets -> sdl_batcher_push_many + sdl_batcher_next "
                                     "(pinned H2D, kernels, D2H of all rows, host batch queue)"}
        res["channel"] = channel_rates(task, cfg, texts)
    return res


def channel_rates(task, cfg, texts, per_record_seconds=3.0):
    """The reference plug-in point (batcher::create_batch, batcher.rs:33-77) fed
    a ProviderChannel stream of the same records: (i) the per-record loop --
    one sdl_batcher_push (a device round trip) per Data message, timed on a
    bounded sample; (ii) create_batch_drained -- every waiting Data message in
    one sdl_batcher_push_many.  Both emit the identical Data sequence
    (tests/test_gpu_drop_in.py)."""
    import queue
    from streaming_data_loader_amd import batcher as Bt

    def stream(recs):
        rx = queue.Queue()
        rx.put(Bt.ProviderChannel.Info("bench"))
        for t in recs:
            rx.put(Bt.ProviderChannel.Data(t))
        rx.put(Bt.ProviderChannel.Complete())
        return rx

    # (i) per record, bounded: records until per_record_seconds have passed
    gt = Bt.GenTokenizer.from_config(cfg)
    gt.create_sync_batch(texts[0])  # warm
    n = done = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < per_record_seconds and n < len(texts):
        gt.create_sync_batch(texts[n])
        done += len(texts[n].encode("utf-8"))
        n += 1
    dt1 = time.perf_counter() - t0
    # (ii) drained: the whole stream waiting in the channel
    total = sum(len(t.encode("utf-8")) for t in texts)
    best = None
    for _ in range(2):
        gt2 = Bt.GenTokenizer.from_config(cfg)
        rx, tx = stream(texts), queue.Queue()
        t0 = time.perf_counter()
        Bt.create_batch_drained(rx, tx, gt2)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
        del tx
    return {"per_record": {"MBps": round(done / dt1 / 1e6, 3), "records": n, "us_per_record": round(dt1 / n * 1e6, 1),
                           "path": "create_batch: one sdl_batcher_push per ProviderChannel::Data"},
            "drained": {"MBps": round(total / best / 1e6, 2), "records": len(texts), "ms": round(best * 1e3, 2),
                        "path": "create_batch_drained: waiting Data messages -> one sdl_batcher_push_many"}}


if __name__ == "__main__":
    main()
