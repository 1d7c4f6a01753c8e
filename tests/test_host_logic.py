"""Host-side logic of the Python mirror (no GPU): the create_batch driver
(rust/src/batcher.rs:33-77), configuration, and the DataSet view."""
import queue

import numpy as np

from streaming_data_loader_amd import batcher as B


class FakeBatcher(B.Batcher):
    """Emits a batch every 2 records; get_working_batch returns a partial one."""

    def __init__(self):
        self.n = 0

    def create_sync_batch(self, data):
        self.n += 1
        return f"batch{self.n}" if self.n % 2 == 0 else None

    def get_working_batch(self):
        return "partial"


def run(msgs):
    rx, tx = queue.Queue(), queue.Queue()
    for m in msgs:
        rx.put(m)
    B.create_batch(rx, tx, FakeBatcher())
    out = []
    while not tx.empty():
        out.append(tx.get())
    return out


def test_create_batch_info_data_complete():
    out = run([B.ProviderChannel.Info({"name": "wiki"}), B.ProviderChannel.Data("a"), B.ProviderChannel.Data("b"),
               B.ProviderChannel.Data("c"), B.ProviderChannel.Complete(), B.ProviderChannel.Data("ignored")])
    assert isinstance(out[0], B.ProviderChannel.Info)
    assert [m.value for m in out[1:3]] == ["batch2", "partial"]
    assert isinstance(out[3], B.ProviderChannel.Complete) and len(out) == 4


def test_channel_close_ends_loop():
    assert run([B.ProviderChannel.Data("a"), None]) == []


def test_mask_length_is_f32_truncation():
    assert [B.get_mask_length(s) for s in (128, 512, 1024)] == [19, 76, 153]


def test_get_case_mirrors_masking_cases():
    c = B.get_case(B.TaskType.Mlm, test=True)
    assert (c.batch.batch_size, c.batch.sequence_length) == (1, 128)
    assert c.dataset_config == B.Mask(19, 103) and c.model_config == B.ModelType.Bert
    c = B.get_case(B.TaskType.Mlm, test=False)
    assert c.batch.batch_size == 4096
    assert B.get_case(B.TaskType.Span, test=False).dataset_config == B.Span(16.0, 2.0)
    assert B.get_case(B.TaskType.MultiLabel, test=False).batch.batch_size == 2048


def test_dataset_to_dict_keys():
    z = np.zeros((2, 4), np.int32)
    d = B.DataSet("bert", 1, z, z + 1, z - 100, z).to_dict()
    assert list(d) == ["input_ids", "attention_mask", "token_type_ids", "labels"]
    assert d["labels"].shape == (1, 4)  # MLM labels list has `index` rows
    g = B.DataSet("gpt2", 2, z, z, z).to_dict()
    assert list(g) == ["input_ids", "attention_mask", "labels"]
