"""util/hash.rs: the oracle and the product's host scalar against the
reference KATs (hash.rs:58-75) and the seeded fixture; the GPU batch against
the same fixture and random batches (gpu-marked)."""
import ctypes

import numpy as np
import pytest

import wal_oracle as W


def _oracle():
    L = W.lib()
    L.oracle_hash.restype = ctypes.c_uint32
    L.oracle_hash.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32]
    L.oracle_hash_batch.restype = None
    L.oracle_hash_batch.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t]
    return L


@pytest.fixture(scope="module")
def hkat():
    import json
    import os
    from conftest import GOLDEN
    with open(os.path.join(GOLDEN, "hash_kat.json")) as f:
        return json.load(f)


def test_oracle_reference_kats(hkat):
    L = _oracle()
    assert len(hkat["kats"]) == 6
    for k in hkat["kats"]:
        d = bytes.fromhex(k["hex"])
        assert L.oracle_hash(d, len(d), k["seed"]) == k["hash"], k["name"]


def test_scalar_matches_kats_and_cases(hkat, arena):
    from lvgpu import hash as H
    for k in hkat["kats"]:
        assert H.hash(bytes.fromhex(k["hex"]), k["seed"]) == k["hash"], k["name"]
    for off, ln, seed, want in hkat["cases"]:
        assert H.hash(arena[off:off + ln], seed) == want
    assert H.cache_shard(0xF0000000) == 15 and H.cache_shard(0x0FFFFFFF) == 0


def _dev(gpu, arr, dtype):
    import torch
    return torch.from_numpy(np.ascontiguousarray(arr).astype(dtype)).to(gpu)


@pytest.mark.gpu
def test_gpu_fixture_cases(gpu, hkat, arena):
    import torch
    from lvgpu import hash as H
    c = np.array(hkat["cases"], dtype=np.uint64)
    a = torch.frombuffer(bytearray(arena), dtype=torch.uint8).to(gpu)
    out = H.hash_batch(a, _dev(gpu, c[:, 0], np.int64), _dev(gpu, c[:, 1], np.int32),
                       _dev(gpu, c[:, 2].astype(np.uint32).view(np.int32), np.int32))
    got = out.cpu().numpy().view(np.uint32)
    assert np.array_equal(got, c[:, 3].astype(np.uint32))
    sh = H.hash_batch(a, _dev(gpu, c[:, 0], np.int64), _dev(gpu, c[:, 1], np.int32),
                      _dev(gpu, c[:, 2].astype(np.uint32).view(np.int32), np.int32), shard=True)
    assert np.array_equal(sh.cpu().numpy().view(np.uint32), c[:, 3].astype(np.uint32) >> 28)


@pytest.mark.gpu
def test_gpu_kats_every_alignment(gpu, hkat):
    import torch
    from lvgpu import hash as H
    offs, lens, seeds, want, buf = [], [], [], [], bytearray()
    for k in hkat["kats"]:
        d = bytes.fromhex(k["hex"])
        for a in range(16):
            buf += bytes(a)
            offs.append(len(buf))
            lens.append(len(d))
            seeds.append(k["seed"])
            want.append(k["hash"])
            buf += d
    buf += bytes(16)
    a = torch.frombuffer(buf, dtype=torch.uint8).to(gpu)
    out = H.hash_batch(a, _dev(gpu, offs, np.int64), _dev(gpu, lens, np.int32),
                       _dev(gpu, np.array(seeds, dtype=np.uint32).view(np.int32), np.int32))
    assert out.cpu().numpy().view(np.uint32).tolist() == want


@pytest.mark.gpu
def test_gpu_random_lengths_and_arena_end(gpu):
    """Every length 0..300 at every offset mod 16, including buffers that end
    at the last byte of the allocation; seeds NULL (cache.rs uses 0)."""
    import torch
    from lvgpu import hash as H
    L = _oracle()
    rng = np.random.default_rng(41)
    size = 1 << 16
    arena = rng.integers(0, 256, size=size, dtype=np.uint8)
    lens = np.repeat(np.arange(0, 301), 16).astype(np.uint32)
    offs = (rng.integers(0, size - 400, size=lens.size) & ~15) + np.tile(np.arange(16), 301)
    offs = np.concatenate([offs, size - np.arange(0, 64)]).astype(np.uint64)
    lens = np.concatenate([lens, np.arange(0, 64)]).astype(np.uint32)
    want = np.zeros(lens.size, dtype=np.uint32)
    L.oracle_hash_batch(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, None, want.ctypes.data, lens.size)
    a = torch.from_numpy(arena).to(gpu)
    out = H.hash_batch(a, _dev(gpu, offs, np.int64), _dev(gpu, lens.view(np.int32), np.int32))
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)


@pytest.mark.gpu
def test_gpu_bad_args(gpu):
    import torch
    from lvgpu import LvError, hash as H
    L = H._bind()
    assert L.lv_hash_batch_device(None, None, None, None, None, 0, 0, None) == 0
    assert L.lv_hash_batch_device(None, None, None, None, None, 5, 0, None) != 0
    a = torch.zeros(16, dtype=torch.uint8, device=gpu)
    with pytest.raises(LvError):
        H.hash_batch(a, torch.zeros(3, dtype=torch.int64, device=gpu), torch.zeros(2, dtype=torch.int32, device=gpu))


@pytest.mark.gpu
def test_gpu_packed_keys_staged_and_not(gpu):
    """Byte-packed keys (the staged-span path: a wave's 64 keys read through
    LDS) of 0..100 B, so some waves hold keys past the 64-B register path and
    some spans exceed the 4 KiB stage; plus a partial last wave and seeds."""
    import torch
    from lvgpu import hash as H
    L = _oracle()
    rng = np.random.default_rng(2718)
    n = 20011
    lens = rng.integers(0, 101, n).astype(np.uint32)
    lens[5000:5064] = rng.integers(60, 101, 64)  # one wave past 4 KiB of span
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    offs += 3  # arena-relative misalignment
    size = int(offs[-1] + lens[-1])
    arena = rng.integers(0, 256, size=size, dtype=np.uint8)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    want = np.zeros(n, dtype=np.uint32)
    L.oracle_hash_batch(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, seeds.ctypes.data,
                        want.ctypes.data, n)
    a = torch.from_numpy(arena).to(gpu)
    out = H.hash_batch(a, _dev(gpu, offs, np.int64), _dev(gpu, lens.view(np.int32), np.int32),
                       _dev(gpu, seeds.view(np.int32), np.int32))
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)


@pytest.mark.gpu
def test_gpu_permuted_and_empty_keys_in_span(gpu):
    """Waves whose keys lie within 4 KiB but out of order (the first lane
    is not the lowest key, the last lane not the highest end), waves whose
    first or last keys are empty, and waves reversed end to end: the kernel
    stages a wave only when every key lies inside the span its first and last
    lanes name, and must hash all of them exactly either way."""
    import torch
    from lvgpu import hash as H
    L = _oracle()
    rng = np.random.default_rng(31337)
    n = 64 * 40 + 17
    lens = rng.integers(0, 65, n).astype(np.uint32)
    lens[0:3] = 0                 # first lanes of wave 0 empty
    lens[64 * 2 - 1] = 0          # last lane of wave 1 empty
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    offs += 5
    for w in range(0, n // 64):
        sl = slice(64 * w, 64 * w + 64)
        if w % 3 == 1:            # shuffled within the wave's span
            p = rng.permutation(64)
            offs[sl], lens[sl] = offs[sl][p], lens[sl][p]
        elif w % 3 == 2:          # reversed: lane 0 holds the highest key
            offs[sl], lens[sl] = offs[sl][::-1].copy(), lens[sl][::-1].copy()
    offs[lens == 0] = rng.integers(0, 4, int((lens == 0).sum()))  # empty keys point anywhere
    size = int((offs + lens).max()) + 1
    arena = rng.integers(0, 256, size=size, dtype=np.uint8)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    want = np.zeros(n, dtype=np.uint32)
    L.oracle_hash_batch(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, seeds.ctypes.data,
                        want.ctypes.data, n)
    a = torch.from_numpy(arena).to(gpu)
    out = H.hash_batch(a, _dev(gpu, offs, np.int64), _dev(gpu, lens.view(np.int32), np.int32),
                       _dev(gpu, seeds.view(np.int32), np.int32))
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)


@pytest.mark.gpu
@pytest.mark.parametrize("width", [4, 8])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 20011])
def test_gpu_packed_bounds(gpu, width, n):
    """lv_hash_batch_packed: key i = arena[b[i], b[i+1]) from n + 1 bounds of
    4 or 8 bytes (lengths from the bound deltas, lane 63 reading the bound
    after its set), empty keys, keys past the 64-B register path and spans
    past the 4 KiB stage, seeded and not, hashes and shards, vs the oracle."""
    import torch
    from lvgpu import hash as H
    L = _oracle()
    rng = np.random.default_rng(n * 10 + width)
    lens = rng.integers(0, 80, n).astype(np.uint32)
    lens[rng.integers(0, n, max(1, n // 50))] = 0
    if n > 5100:
        lens[5000:5064] = rng.integers(70, 101, 64)
    bounds = np.zeros(n + 1, dtype=np.uint64)
    bounds[1:] = np.cumsum(lens, dtype=np.uint64)
    bounds += 7
    arena = rng.integers(0, 256, size=int(bounds[-1]) + 3, dtype=np.uint8)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    offs = bounds[:-1].copy()
    a = torch.from_numpy(arena).to(gpu)
    b = _dev(gpu, bounds, np.int32 if width == 4 else np.int64)
    for sd in (None, seeds):
        want = np.zeros(n, dtype=np.uint32)
        L.oracle_hash_batch(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                            None if sd is None else sd.ctypes.data, want.ctypes.data, n)
        ds = None if sd is None else _dev(gpu, sd.view(np.int32), np.int32)
        got = H.hash_batch_packed(a, b, ds).cpu().numpy().view(np.uint32)
        assert np.array_equal(got, want)
        sh = H.hash_batch_packed(a, b, ds, shard=True).cpu().numpy().view(np.uint32)
        assert np.array_equal(sh, want >> 28)


@pytest.mark.gpu
def test_gpu_packed_bad_args(gpu):
    import torch
    from lvgpu import hash as H
    L = H._bind()
    assert L.lv_hash_batch_packed(None, None, 8, None, None, 0, 0, None) == 0
    a = torch.zeros(16, dtype=torch.uint8, device=gpu)
    b = torch.zeros(3, dtype=torch.int64, device=gpu)
    o = torch.zeros(2, dtype=torch.int32, device=gpu)
    assert L.lv_hash_batch_packed(a.data_ptr(), b.data_ptr(), 2, None, o.data_ptr(), 2, 0, None) != 0
    assert L.lv_hash_batch_packed(a.data_ptr(), b.data_ptr() + 4, 8, None, o.data_ptr(), 2, 0, None) != 0
