"""The drop-in boundary at the reference's plug-in point, on the GPU.

batcher::create_batch (batcher.rs:33-77) calls create_sync_batch once per
ProviderChannel::Data: through the C ABI that is one device round trip per
record (sdl_batcher_push).  create_batch_drained hands every Data message
already waiting in the channel to ONE sdl_batcher_push_many call.  These tests
check that the drained loop sends the identical message sequence (every Data
batch's planes and row count, Info in stream order, the one flushed batch,
Complete) as the per-record loop, for every task and for the B=1 case where
the reference's cadence drops queued batches.  Also: `bench.py --gpus 1
--spawn` (the rank launcher) reports n_gpus == 1."""
import json
import os
import queue
import subprocess
import sys

import numpy as np
import pytest

from streaming_data_loader_amd import arrow_io
from streaming_data_loader_amd import batcher as B
from streaming_data_loader_amd import native

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")


def stream(records, info_at=(0, 20)):
    """A provider stream: Info at the given positions, one Data per record, Complete."""
    msgs = []
    for i, r in enumerate(records):
        if i in info_at:
            msgs.append(B.ProviderChannel.Info(f"info@{i}"))
        msgs.append(B.ProviderChannel.Data(r))
    msgs.append(B.ProviderChannel.Complete())
    return msgs


def run_loop(loop, make, msgs, **kw):
    rx, tx = queue.Queue(), queue.Queue()
    for m in msgs:
        rx.put(m)
    loop(rx, tx, make(), **kw)
    out = []
    while not tx.empty():
        m = tx.get()
        if isinstance(m, B.ProviderChannel.Data):
            d = m.value
            out.append(("data", d.rows, d.input_ids.copy(), d.attention_mask.copy(),
                        None if d.token_type_ids is None else d.token_type_ids.copy(), d.labels.copy()))
        elif isinstance(m, B.ProviderChannel.Info):
            out.append(("info", m.value))
        else:
            out.append(("complete",))
    return out


def assert_same(a, b):
    assert [x[0] for x in a] == [x[0] for x in b]
    for x, y in zip(a, b):
        if x[0] == "info":
            assert x == y
        elif x[0] == "data":
            assert x[1] == y[1]
            for u, v in zip(x[2:], y[2:]):
                if u is None:
                    assert v is None
                else:
                    np.testing.assert_array_equal(u, v)


CASES = {
    "mlm-b4": lambda: B.GenTokenizer(B.ModelType.Bert, B.BatchConfig(4, 128), B.Mask(19, 103), B.TokenizerConfig(),
                                     seed=11),
    "mlm-b1": lambda: B.GenTokenizer(B.ModelType.Bert, B.BatchConfig(1, 128), B.Mask(19, 103), B.TokenizerConfig(),
                                     seed=12),
    "clm-b4": lambda: B.GenTokenizer.from_config(B.get_case(B.TaskType.Clm, False, 256, 4, 13)),
    "span-b4": lambda: B.GenTokenizer.from_config(B.get_case(B.TaskType.Span, False, 128, 4, 14)),
}


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("max_bytes", [64 << 20, 3000])
def test_drained_loop_sends_the_per_record_sequence(native_lib, records, case, max_bytes):
    msgs = stream(records * 2)
    one = run_loop(B.create_batch, CASES[case], msgs)
    many = run_loop(B.create_batch_drained, CASES[case], msgs, max_bytes=max_bytes)
    assert sum(1 for x in one if x[0] == "data") > 1
    assert_same(one, many)


def test_drained_loop_with_a_live_producer(native_lib, records):
    """Records arriving while the Batcher runs: drains of every size, same sequence."""
    import threading
    import time
    msgs = stream(records * 3, info_at=(0, 7, 64))
    one = run_loop(B.create_batch, CASES["mlm-b4"], msgs)
    rx, tx = queue.Queue(), queue.Queue()

    def produce():
        for i, m in enumerate(msgs):
            rx.put(m)
            if i % 5 == 0:
                time.sleep(0.002)

    th = threading.Thread(target=produce)
    th.start()
    B.create_batch_drained(rx, tx, CASES["mlm-b4"]())
    th.join()
    many = []
    while not tx.empty():
        m = tx.get()
        if isinstance(m, B.ProviderChannel.Data):
            d = m.value
            many.append(("data", d.rows, d.input_ids.copy(), d.attention_mask.copy(), d.token_type_ids.copy(),
                         d.labels.copy()))
        elif isinstance(m, B.ProviderChannel.Info):
            many.append(("info", m.value))
        else:
            many.append(("complete",))
    assert_same(one, many)


def test_drained_simple_batcher_multi_label(native_lib):
    """SimpleBatcher (S = SimpleTransport, simple_batcher.rs:31-53) from the Arrow fixture."""
    items = []
    for b in arrow_io.read_stream(os.path.join(GOLDEN, "multi_label.arrow")):
        gen = arrow_io.MultiArrowGenerator(b.schema)
        items += [gen.get_data(b, i) for i in range(b.num_rows)]
    make = lambda: B.SimpleBatcher(B.ModelType.Bert, B.MultiLabel(9), B.BatchConfig(8, 128),  # noqa: E731
                                   B.TokenizerConfig())
    msgs = stream(items, info_at=(0, 5))
    one = run_loop(B.create_batch, make, msgs)
    many = run_loop(B.create_batch_drained, make, msgs, max_bytes=2000)
    assert_same(one, many)


def test_bench_spawn_path_reports_one_gpu(native_lib):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, "-u", os.path.join(REPO, "bench.py"), "--gpus", "1", "--spawn", "--steps", "2",
                        "--warmup", "1", "--arena-mib", "8", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=110, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["errors"] == {"tokenize": 0, "label": 0}
    # the held-out leg rides along with a fixture run, beside `value`
    h = d["heldout"]
    assert h["value"] > 0 and h["errors"] == {"tokenize": 0, "label": 0} and h["roofline"]["avg_launch_ms"] > 0
