import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "leveldb-rs_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs under gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def kat():
    with open(os.path.join(GOLDEN, "crc32c_kat.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def wal_golden():
    with open(os.path.join(GOLDEN, "wal_scenarios.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def arena(kat):
    """The 1 MiB splitmix64 arena the random golden cases index into."""
    import ctypes
    import hashlib

    import wal_oracle as W
    a = kat["arena"]
    buf = ctypes.create_string_buffer(a["bytes"])
    W.lib().oracle_fill_splitmix(buf, 0, a["bytes"], a["seed"])
    raw = buf.raw
    assert hashlib.sha256(raw).hexdigest() == a["sha256"]
    return raw


def kat_bytes(k):
    if k["hex"] is not None:
        return bytes.fromhex(k["hex"])
    return bytes([k["fill"]["byte"]]) * k["fill"]["n"]


@pytest.fixture(scope="session")
def gpu():
    """Skip unless a GPU is visible; on a GPU box, the HIP library must load."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import lvgpu
    lvgpu.device_init()
    return torch.device("cuda:0")
