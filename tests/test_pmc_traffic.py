"""bench.py's HBM traffic accounting (DESIGN.md §4 "Traffic accounting (r04)").

The text + offsets stream counts at its own bytes, the calibrated share of FETCH_SIZE
(the load-only build's FETCH_SIZE per stream byte, profiles/pmc/stream_calibration.json)
comes out of the kernel's FETCH_SIZE, the rest is added as reported, with WRITE_SIZE.
Checked on a synthetic summary and on every committed r04 summary."""
import json
import re
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_split_arithmetic():
    cal = bench.stream_calibration()
    assert cal is not None and 0.5 <= cal["ratio"] <= 1.0
    stream = 1_000_000
    pmc = {"counters": {"FETCH_SIZE": (cal["ratio"] * stream + 50_000) / 1024, "WRITE_SIZE": 300_000 / 1024}}
    traffic, split = bench.pmc_traffic(pmc, stream)
    assert split["stream_read"] == stream
    assert abs(split["probe_and_list_read"] - 50_000) <= 2
    assert abs(split["write"] - 300_000) <= 1
    assert abs(traffic - (stream + 50_000 + 300_000)) <= 3
    assert split["uniform_x2_upper_bound"] >= traffic
    # FETCH_SIZE below the calibrated stream share: nothing negative is added
    low = {"counters": {"FETCH_SIZE": 10.0, "WRITE_SIZE": 0.0}}
    t2, s2 = bench.pmc_traffic(low, stream)
    assert s2["probe_and_list_read"] == 0 and t2 == stream


def test_calibration_matches_the_bench_arena():
    cal = bench.stream_calibration()
    _, _, offs, _, _ = bench.shard(0, cal["arena_mib"] << 20, "fixture", 1)
    assert cal["text_bytes"] == int(offs[-1]) and cal["records"] == len(offs) - 1
    assert cal["stream_bytes"] == int(offs[-1]) + 8 * len(offs)


@pytest.mark.parametrize("task,kernel", [("mlm", "k_wordpiece_chunks"), ("clm", "k_bpe_chunks"),
                                         ("span", "k_unigram_chunks"), ("multi-label", "k_wordpiece_chunks"),
                                         ("single-class", "k_wordpiece_chunks")])
def test_committed_summaries_give_a_split(task, kernel):
    pmc, note = bench.load_pmc(task, 256, kernel, "fixture")
    assert pmc is not None, note
    cal = bench.stream_calibration()
    traffic, split = bench.pmc_traffic(pmc, cal["stream_bytes"])
    # at least the stream and the writes; never above the old uniform x2 reading
    assert split["stream_read"] + split["write"] <= traffic <= split["uniform_x2_upper_bound"]
    with open(os.path.join(REPO, "profiles", "pmc", f"{task}_256mib.json")) as f:
        assert re.search(r"\(r0[4-9]\)", json.load(f).get("date", ""))  # (a dated, current-round summary)


@pytest.mark.parametrize("task", ["span", "clm"])
def test_stage_counters_sum_every_launch(task):
    """span and clm time their whole tokenize stage (the chunk kernel plus the Viterbi / long-item
    launches): their PMC figures are the sum over those launches' per-launch counters."""
    kernels = bench.TASKS[task]["pmc_kernels"]
    pmc, note = bench.load_pmc(task, 256, kernels, "fixture")
    assert pmc is not None, note
    with open(os.path.join(REPO, "profiles", "pmc", f"{task}_256mib.json")) as f:
        d = json.load(f)
    names = [n for n in d["kernels"] for k in kernels if n == "sdl::" + k or n.startswith("sdl::" + k + "<")]
    assert len(names) >= 2 and sorted(pmc["kernels_summed"]) == sorted(n.replace("sdl::", "") for n in names)
    for c in ("SQ_INSTS_VALU", "FETCH_SIZE", "WRITE_SIZE"):
        want = sum(d["kernels"][n]["counters"].get(c, 0.0) for n in names)
        assert abs(pmc["counters"][c] - want) <= 1e-6 * max(want, 1.0)
    # a single kernel name still returns that kernel's own entry
    one, _ = bench.load_pmc(task, 256, bench.TASKS[task]["kernel"], "fixture")
    assert "kernels_summed" not in one
