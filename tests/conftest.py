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


def gpu_selected(config) -> bool:
    """True when the run selects the gpu marker (`-m gpu`, `-m "gpu and ..."`):
    a GPU run, where a missing device is a failure, not a skip."""
    expr = (config.getoption("markexpr", default="") or "").replace("(", " ").replace(")", " ").split()
    return any(tok == "gpu" and (i == 0 or expr[i - 1] != "not") for i, tok in enumerate(expr))


@pytest.fixture(scope="session")
def gpu(request):
    """The GPU every `gpu` test runs on.  Under `-m gpu` a missing device
    FAILS the test (a GPU run that executes nothing must not look green);
    otherwise (a plain `pytest` on a CPU host) the test is skipped.  On a GPU
    box the HIP library must load."""
    import torch
    if not torch.cuda.is_available():
        msg = "no GPU visible (torch.cuda.is_available() is False)"
        if gpu_selected(request.config):
            pytest.fail(msg + " in a run that selects -m gpu", pytrace=False)
        pytest.skip(msg)
    import lvgpu
    lvgpu.device_init()
    return torch.device("cuda:0")
