"""Randomised parity sweep of the device WAL scan (lv_wal_scan_device)
against the oracle's
framing of log_reader.rs:271-331 (oracle.scan_log).  Each trial draws a log
from one generator: 1-3,000 records of log-uniform sizes up to 2^8-2^16
bytes (fragmented by the oracle Writer, log_writer.rs:67-80) after a random
dest_length, then some of: flipped payload and header bytes, headers forced
to ZERO or to a length past the block, a truncated tail, zero padding or
random garbage appended; the log placed 8-B or 16-B aligned in HBM; the
capacity exact, larger or one short (count reported, nothing written).
Every offset, info word and CRC is compared with the oracle.
LVGPU_WAL_STRESS_TRIALS sets the number of trials (default 24)."""
import os

import numpy as np
import pytest

import wal_oracle as W

pytestmark = pytest.mark.gpu
B, H = W.BLOCK_SIZE, W.HEADER_SIZE
TRIALS = int(os.environ.get("LVGPU_WAL_STRESS_TRIALS", "24"))
SORTED = "wal_hist+sort_scan+wal_scatter+crc32c_classes_kernel"


def _log(rng):
    n = int(rng.integers(1, 3001))
    maxlog = int(rng.integers(8, 17))
    recs = []
    for _ in range(n):
        ln = int(rng.integers(0, 1 << int(rng.integers(0, maxlog + 1))))
        recs.append(rng.integers(0, 256, size=ln, dtype=np.uint8).tobytes())
    d = bytearray()
    w = W.Writer(d, int(rng.integers(0, 2 * B)))
    for r in recs:
        w.add_record(r)
    log = bytearray(d)
    if len(log) and rng.random() < 0.5:  # flipped bytes anywhere (payloads and headers)
        for p in rng.integers(0, len(log), size=int(rng.integers(1, 40))):
            log[int(p)] ^= int(rng.integers(1, 256))
    nblk = len(log) // B
    if nblk and rng.random() < 0.3:  # a ZERO header / a length past the block, at a block start
        b = int(rng.integers(0, nblk)) * B
        if rng.random() < 0.5:
            log[b + 4:b + 7] = bytes(3)
        else:
            log[b + 4:b + 6] = int(rng.integers(B - H + 1, 65536)).to_bytes(2, "little")
    if len(log) and rng.random() < 0.3:  # a truncated tail (possibly inside a header)
        del log[len(log) - int(rng.integers(1, min(len(log), 3 * B) + 1)):]
    r = rng.random()
    if r < 0.15:
        log += bytes(int(rng.integers(1, 3 * B)))  # a preallocated zero tail
    elif r < 0.25:
        log += rng.integers(0, 256, size=int(rng.integers(1, 3 * B)), dtype=np.uint8).tobytes()
    return bytes(log)


@pytest.mark.parametrize("trial", range(TRIALS))
def test_wal_scan_device_random(gpu, trial):
    import torch

    import lvgpu
    import lvgpu.wal as LW
    rng = np.random.default_rng(53_000 + trial)
    log = _log(rng)
    o, c, i = W.scan_log(log)
    n = len(o)
    cap = [n, n + int(rng.integers(1, 100)), max(n - 1, 0)][int(rng.integers(0, 3))]
    shift = int(rng.choice([0, 8]))
    t = torch.frombuffer(bytearray(bytes(shift) + log + b"\0"), dtype=torch.uint8).to(gpu)[shift:shift + len(log)]
    kern = SORTED + ("+wal_unsort" if cap else "")
    hdr, crc, info, count = LW.scan_device(t, cap)
    torch.cuda.synchronize()
    assert lvgpu.last_kernel() == kern or len(log) == 0, (trial, lvgpu.last_kernel())
    got = int(count.item())
    assert got == n, (trial, got, n)
    if n <= cap:
        assert hdr[:n].cpu().numpy().tolist() == o, trial
        assert info[:n].cpu().numpy().view(np.uint32).tolist() == i, trial
        assert crc[:n].cpu().numpy().view(np.uint32).tolist() == c, trial
