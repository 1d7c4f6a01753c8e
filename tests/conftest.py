import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def records():
    with open(os.path.join(GOLDEN, "test_records.jsonl"), encoding="utf-8") as f:
        return [json.loads(l)["text"] for l in f]


@pytest.fixture(scope="session")
def bert_goldens():
    with open(os.path.join(GOLDEN, "bert_ids.json"), encoding="utf-8") as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle_tok():
    import oracle_lib
    return oracle_lib.Tok()


@pytest.fixture(scope="session")
def native_lib():
    from streaming_data_loader_amd import build, native
    build.build()
    return native.load()


@pytest.fixture(scope="session")
def gpt2_goldens():
    with open(os.path.join(GOLDEN, "gpt2_ids.json"), encoding="utf-8") as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle_gpt2():
    import oracle_lib
    return oracle_lib.Gpt2Tok()
