"""Randomised parity sweep of the device offsets API (lv_crc32c_batch_device
and lv_crc32c_batch_device_ws) against the oracle: every path the library
picks for a batch -- the fused small-batch kernel (n <= 1,024, local and
straddling split buffers), the length sort + class kernel (n > 1,024, one-key
batches, split long buffers joined by combine_long_kernel) -- on batches
drawn from one generator: buffer counts 1-6,000, lengths from empty to 8 MiB
in a mix of size classes, byte-packed, 256-B-aligned or overlapping offsets,
seeded or not, masked or not, library or caller workspace, with or without
the exact host-side length hint (lv_crc32c_batch_device_hint, whose join
decision is checked against the kernels it launched).  Every output is
checked bit-exact (the C restatement of crc32c.rs in oracle/).
LVGPU_STRESS_TRIALS sets the number of trials (default 40)."""
import ctypes
import os

import numpy as np
import pytest

import lvgpu
from test_gpu_batch import oracle_batch

pytestmark = pytest.mark.gpu
ARENA_BUDGET = 256 << 20  # bytes of payload per trial (the oracle checks all of it on the host)


@pytest.fixture(scope="module")
def torch_dev(gpu):
    import torch
    return torch, gpu


CLASSES = [(0, 1), (1, 129), (129, 1025), (1025, 16385), (16385, 65537), (65537, 1 << 20), (1 << 20, 8 << 20)]


def _batch(rng):
    n = int(rng.choice([1, 2, 7, 100, 1000, 1024, 1025, 3000, 6000]))
    w = rng.dirichlet(np.ones(len(CLASSES)) * 0.7)
    w[-1] *= 0.05 if n > 64 else 1.0  # keep the arena small: few multi-MiB buffers in big batches
    w /= w.sum()
    cls = rng.choice(len(CLASSES), size=n, p=w)
    lens = np.array([int(rng.integers(*CLASSES[c])) for c in cls], dtype=np.int64)
    while lens.sum() > ARENA_BUDGET:  # shrink the long ones (those above 64 KiB first)
        lens[lens > (65536 if (lens > 65536).any() else 4096)] //= 2
    layout = rng.choice(["packed", "aligned", "overlap"])
    if layout == "overlap":
        span = int(lens.max()) + 4096
        offs = np.array([int(rng.integers(0, span - int(l) + 1)) for l in lens], dtype=np.int64)
        end = span
    else:
        offs, pos = [], int(rng.integers(0, 16))
        for l in lens:
            offs.append(pos)
            pos += int(l) + int(rng.integers(0, 9))
            if layout == "aligned":
                pos = (pos + 255) & ~255
        offs, end = np.array(offs, dtype=np.int64), pos
    return lens, offs, end, layout


TRIALS = int(os.environ.get("LVGPU_STRESS_TRIALS", "40"))


@pytest.mark.parametrize("trial", range(TRIALS))
def test_offsets_api_random_sweep(torch_dev, trial):
    torch, dev = torch_dev
    rng = np.random.default_rng(77_000 + trial)
    lens, offs, end, layout = _batch(rng)
    n = lens.size
    arena = torch.empty(end + 64, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(arena, 0, 0x57E55 + trial)
    seeded, masked, caller = bool(rng.integers(0, 2)), bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
    seeds = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32) if seeded else None
    o = torch.from_numpy(offs).to(dev)
    ln = torch.from_numpy(lens.astype(np.int32)).to(dev)
    sd = None if seeds is None else torch.from_numpy(seeds.view(np.int32)).to(dev)
    hinted = bool(np.random.default_rng(91_000 + trial).integers(0, 2))  # (its own stream: the batches stay round 3's)
    ws = torch.full((lvgpu.workspace_bytes(n),), 0xA5, dtype=torch.uint8, device=dev) if caller else None
    if hinted:
        hint = lvgpu.hint_for(lens)
        out = lvgpu.batch_hint(arena, o, ln, hint, seed=sd, masked=masked, workspace=ws)
    elif caller:
        out = lvgpu.batch_ws(arena, o, ln, ws, sd, masked=masked)
    else:
        out = lvgpu.batch(arena, o, ln, sd, masked=masked)
    kern = lvgpu.last_kernel()
    base = "crc32c_fused_small_kernel" if n <= 1024 else "sort+crc32c_classes_kernel"
    join = True
    if hinted:
        L = lvgpu.lib()
        L.lv_crc32c_hint_needs_join.restype = ctypes.c_int
        L.lv_crc32c_hint_needs_join.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
        join = bool(L.lv_crc32c_hint_needs_join(ctypes.addressof(hint), n,
                                                torch.cuda.get_device_properties(dev).multi_processor_count))
    if hinted and n > 1024 and hint.uniform and not join:
        base = "hint_len_kernel+crc32c_classes_kernel"  # host-known identity list: no sort
    assert kern == base + ("+combine_long_kernel" if join else ""), (kern, hinted)
    got = out.cpu().numpy().view(np.uint32)
    want = oracle_batch(arena.cpu().numpy().tobytes(), offs, lens, seeds, masked)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (n, layout, seeded, masked, caller, hinted, [(int(i), int(lens[i])) for i in bad[:8]])
