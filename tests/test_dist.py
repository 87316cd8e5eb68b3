"""Multi-rank path on CPU (gloo, world_size 2): sharding by bytes covers every
buffer exactly once, and per-rank checksums gathered over the process group
equal the single-process result.  The per-rank checksum here is the CPU oracle
(the GPU kernel is covered by the gpu tests); what is under test is the shard
assignment and the gather, i.e. the N>1 host logic of bench.py."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from lvgpu.shard import shard_bounds, uniform_bounds


def test_shard_bounds_cover_and_balance():
    rng = np.random.default_rng(5)
    ln = (32 * np.minimum(rng.zipf(1.1, size=50000), 2048)).astype(np.uint32)
    for world in (1, 2, 3, 8):
        b = shard_bounds(ln, world)
        assert b[0] == 0 and b[-1] == ln.size and all(b[i] <= b[i + 1] for i in range(world))
        shares = [int(ln[b[r]:b[r + 1]].sum(dtype=np.uint64)) for r in range(world)]
        assert sum(shares) == int(ln.sum(dtype=np.uint64))
        assert max(shares) - min(shares) <= 2 * int(ln.max())  # within one buffer of even
    assert shard_bounds([], 4) == [0, 0, 0, 0, 0]
    assert uniform_bounds(10, 4) == [0, 2, 5, 7, 10]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, arena, offs, lens, result_path):
    import torch
    import torch.distributed as dist
    import wal_oracle as W
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = shard_bounds(lens, world)
    lo, hi = b[rank], b[rank + 1]
    mine = np.array([W.extend(0, arena[offs[i]:offs[i] + lens[i]]) for i in range(lo, hi)], dtype=np.int64)
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([mine.size], dtype=torch.int64))
    maxn = int(max(s.item() for s in sizes))
    pad = torch.zeros(maxn, dtype=torch.int64)
    pad[: mine.size] = torch.from_numpy(mine)
    gathered = [torch.zeros(maxn, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(gathered, pad)
    if rank == 0:
        full = np.concatenate([g[: int(s.item())].numpy() for g, s in zip(gathered, sizes)])
        np.save(result_path, full)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_shards(tmp_path):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (os.path.join(root, "oracle"), os.path.join(root, "leveldb-rs_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import wal_oracle as W
    rng = np.random.default_rng(9)
    lens = (rng.integers(0, 3000, size=400)).astype(np.uint32)
    offs = np.zeros(lens.size, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    arena = rng.integers(0, 256, size=int(lens.sum()) + 16, dtype=np.uint8).tobytes()
    out = str(tmp_path / "crcs.npy")
    mp.spawn(_worker, args=(2, _free_port(), arena, offs.tolist(), lens.tolist(), out), nprocs=2, join=True)
    got = np.load(out)
    want = np.array([W.extend(0, arena[int(offs[i]):int(offs[i]) + int(lens[i])]) for i in range(lens.size)],
                    dtype=np.int64)
    assert np.array_equal(got, want)
