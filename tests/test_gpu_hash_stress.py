"""Randomised parity sweep of the batched hash (util/hash.rs:20-51) against
the oracle: each trial draws 1-60,000 keys with lengths from one of several
mixes (tiny 0-8 B, cache-key-like 8-64 B, 0-300 B, a few of 1-5 KiB among
short ones), laid out byte-packed, 16-B aligned, shuffled over the arena or
overlapping, at a random arena misalignment, seeded or not; hashes and cache
shards through lv_hash_batch_device, and for byte-packed layouts through
lv_hash_batch_packed with 4- and 8-byte bounds.  Bit-exact.
LVGPU_HASH_STRESS_TRIALS sets the number of trials (default 12)."""
import ctypes
import os

import numpy as np
import pytest

import wal_oracle as W

pytestmark = pytest.mark.gpu
TRIALS = int(os.environ.get("LVGPU_HASH_STRESS_TRIALS", "12"))


def _oracle():
    L = W.lib()
    L.oracle_hash_batch.restype = None
    L.oracle_hash_batch.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t]
    return L


def _dev(gpu, a, dt):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(gpu)


def _lens(rng, n):
    mix = int(rng.integers(0, 4))
    if mix == 0:
        lens = rng.integers(0, 9, n)
    elif mix == 1:
        lens = rng.integers(8, 65, n)
    elif mix == 2:
        lens = rng.integers(0, 301, n)
    else:
        lens = rng.integers(0, 40, n)
        lens[rng.integers(0, n, max(1, n // 200))] = rng.integers(1024, 5121, max(1, n // 200))
    return lens.astype(np.uint32)


@pytest.mark.parametrize("trial", range(TRIALS))
def test_hash_random(gpu, trial):
    from lvgpu import hash as H
    import torch
    L = _oracle()
    rng = np.random.default_rng(67_000 + trial)
    n = int(rng.choice([1, 63, 64, 65, 1000, int(rng.integers(1, 60001))]))
    lens = _lens(rng, n)
    lay = int(rng.integers(0, 4))  # 0 packed, 1 16-B aligned, 2 shuffled packed, 3 overlapping
    mis = int(rng.integers(0, 16))
    if lay in (0, 2):
        offs = np.zeros(n, dtype=np.uint64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        size = int(lens.sum())
    elif lay == 1:
        al = (lens.astype(np.uint64) + 15) & ~np.uint64(15)
        offs = np.zeros(n, dtype=np.uint64)
        offs[1:] = np.cumsum(al[:-1], dtype=np.uint64)
        size = int(al.sum())
    else:
        size = int(lens.max()) * 4 + 64
        offs = rng.integers(0, size - int(lens.max()) + 1, n).astype(np.uint64)
    packed = lay == 0
    if lay == 2:
        perm = rng.permutation(n)
        offs, lens = offs[perm], lens[perm]
    offs = offs + mis
    arena = rng.integers(0, 256, size=size + mis + 16, dtype=np.uint8)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) if rng.random() < 0.5 else None
    want = np.zeros(n, dtype=np.uint32)
    L.oracle_hash_batch(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                        None if seeds is None else seeds.ctypes.data, want.ctypes.data, n)
    a = torch.from_numpy(arena).to(gpu)
    ds = None if seeds is None else _dev(gpu, seeds, np.int32)
    got = H.hash_batch(a, _dev(gpu, offs, np.int64), _dev(gpu, lens, np.int32), ds).cpu().numpy().view(np.uint32)
    assert np.array_equal(got, want), trial
    sh = H.hash_batch(a, _dev(gpu, offs, np.int64), _dev(gpu, lens, np.int32), ds, shard=True)
    assert np.array_equal(sh.cpu().numpy().view(np.uint32), want >> 28), trial
    if packed:
        bounds = np.concatenate([offs, [offs[-1] + lens[-1]]]).astype(np.uint64)
        for dt in (np.int32, np.int64):
            b = _dev(gpu, bounds.astype(np.uint32) if dt is np.int32 else bounds, dt)
            got = H.hash_batch_packed(a, b, ds).cpu().numpy().view(np.uint32)
            assert np.array_equal(got, want), (trial, dt)
