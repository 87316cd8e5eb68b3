"""Randomised parity sweep of the SSTable trailer kernels (seal and verify,
include/lvgpu/table.h) against the oracle trailer (oracle/table_oracle.py;
the trailer layout itself is parity-unpinned, see table.h).  Each trial
draws a table of 1-2,500 blocks (<= 400 when sizes are mixed) with sizes
from one of several mixes (all 4 KiB-ish as a table builder makes them,
mixed 0-70,000 B, tiny 0-40 B),
handles in file order or shuffled, per-block types or none; seals it on the
device and compares every byte with the oracle's seal; then corrupts some
blocks (contents, type or stored CRC), adds handles past the end or
overflowing, and compares every verify status and CRC with the oracle's.
LVGPU_SST_STRESS_TRIALS sets the number of trials (default 12)."""
import os

import numpy as np
import pytest

import table_oracle as T
import wal_oracle as W
from test_table import _make_table, _oracle_seal

pytestmark = pytest.mark.gpu
TRIALS = int(os.environ.get("LVGPU_SST_STRESS_TRIALS", "12"))


def _sizes(rng, n):
    mix = int(rng.integers(0, 3))
    if mix == 0:
        return 4096 + rng.integers(0, 256, size=n)
    if mix == 1:
        return rng.integers(0, 70000, size=n)
    return rng.integers(0, 41, size=n)


@pytest.mark.parametrize("trial", range(TRIALS))
def test_sst_seal_verify_random(gpu, trial):
    import torch
    from lvgpu import table as LT
    rng = np.random.default_rng(61_000 + trial)
    n = int(rng.integers(1, 2501))
    sizes = _sizes(rng, n)
    if sizes.max(initial=0) > 8192:
        n = min(n, 400)  # mixed sizes up to 70 KB: <= ~28 MB of table, so a trial stays ~1 s
        sizes = sizes[:n]
    file, handles = _make_table(rng, n, sizes=sizes)
    if rng.random() < 0.5:
        handles = [handles[i] for i in rng.permutation(n)]
    typed = rng.random() < 0.5
    types = rng.integers(0, 256, size=n).astype(np.uint8) if typed else np.zeros(n, dtype=np.uint8)
    d = torch.frombuffer(bytearray(file), dtype=torch.uint8).to(gpu)
    h = torch.tensor(handles, dtype=torch.int64, device=gpu)
    LT.seal_blocks(d, h, torch.from_numpy(types).to(gpu) if typed else None)
    want = _oracle_seal(file, handles, types.tolist())
    assert d.cpu().numpy().tobytes() == want, trial
    sealed = bytearray(want)
    for k in sorted(set(int(x) for x in rng.integers(0, n, size=int(rng.integers(0, 30))))):
        o, sz = handles[k]
        sealed[o + int(rng.integers(0, sz + 5))] ^= int(rng.integers(1, 256))
    extra = [(len(sealed) - 4, 0), (len(sealed), 0), (2**63, 1), (0, 2**40)][:int(rng.integers(0, 5))]
    allh = handles + extra
    sb = bytes(sealed)
    want_st = [T.verify_block(sb, T.BlockHandle(o, s)) for o, s in allh]
    d = torch.frombuffer(bytearray(sb), dtype=torch.uint8).to(gpu)
    hh = torch.tensor(np.array(allh, dtype=np.uint64).view(np.int64), device=gpu)
    st, crc = LT.verify_blocks(d, hh, out_crc=True)
    assert st.cpu().numpy().tolist() == want_st, trial
    got = crc.cpu().numpy().view(np.uint32).tolist()
    for (o, s), c, w in zip(allh, got, want_st):
        if w != 2:  # in range: crc32c(contents || type) of the (possibly corrupted) bytes
            assert c == W.value(sb[o:o + s + 1]), trial
    assert LT.verify_blocks(d, hh).cpu().numpy().tolist() == want_st, trial
