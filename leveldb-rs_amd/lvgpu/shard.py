"""Sharding of a batch across GPUs (one process per GPU, torch.distributed).

Buffers are independent, so a batch splits into contiguous index ranges, one
per rank, with no data-path collective.  Ranges are
balanced by payload bytes (a prefix sum of the lengths), not by count, so a
Zipf mix of 32 B records and 64 KiB blocks still loads every GPU equally;
fixed-size blocks (C3/C5) split by count.

The functions below are the whole N > 1 host logic of `bench.py`: the
rank's range of a global batch (`RankShard`), the timed region between
barriers with the max over ranks (`timed_steps`), and the gather of per-rank
figures into the aggregate (`gather_ranks`, `aggregate`).  The world-size-2
gloo test (tests/test_dist.py) drives the same functions with the CPU oracle
as the per-rank compute.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import numpy as np


def shard_bounds(lengths, world: int):
    """Start index of each rank's range (len world+1): rank r owns
    [b[r], b[r+1]).  Each range holds ~1/world of the total bytes; ties and
    zero-length buffers go to the lower rank."""
    if world < 1:
        raise ValueError("world must be >= 1")
    ln = np.asarray(lengths, dtype=np.uint64)
    n = ln.size
    if n == 0:
        return [0] * (world + 1)
    csum = np.cumsum(ln, dtype=np.uint64)
    total = int(csum[-1])
    bounds = [0]
    for r in range(1, world):
        target = (total * r) // world
        # first index whose inclusive prefix exceeds the target
        bounds.append(int(np.searchsorted(csum, target, side="right")))
    bounds.append(n)
    for r in range(1, world + 1):  # monotone
        bounds[r] = max(bounds[r], bounds[r - 1])
    return bounds


def uniform_bounds(n: int, world: int):
    """Equal-count ranges for fixed-size blocks (C3/C5)."""
    return [(n * r) // world for r in range(world + 1)]


@dataclass
class RankShard:
    """Rank `rank`'s contiguous slice [lo, hi) of a global batch whose buffers
    are byte-packed (or strided) in ONE global arena.  The rank materialises
    only the arena bytes [byte_lo, byte_hi) of its slice; `local_off` are its
    buffers' offsets rebased to that span, `lens` their lengths.  A rank's
    results are out[lo:hi] of the global output."""
    rank: int
    world: int
    lo: int
    hi: int
    byte_lo: int
    byte_hi: int
    local_off: np.ndarray  # uint64
    lens: np.ndarray       # uint32

    @property
    def n(self) -> int:
        return self.hi - self.lo

    @property
    def payload_bytes(self) -> int:
        return int(self.lens.sum(dtype=np.uint64))

    @staticmethod
    def uniform(n_total: int, block: int, rank: int, world: int) -> "RankShard":
        """Fixed-size blocks at offsets i*block (C3/C5), split by count."""
        b = uniform_bounds(n_total, world)
        lo, hi = b[rank], b[rank + 1]
        off = np.arange(hi - lo, dtype=np.uint64) * np.uint64(block)
        return RankShard(rank, world, lo, hi, lo * block, hi * block, off,
                         np.full(hi - lo, block, dtype=np.uint32))

    @staticmethod
    def packed(lengths, rank: int, world: int) -> "RankShard":
        """Byte-packed buffers (global offset of buffer i = sum of the lengths
        before it: C2/C4), split by payload bytes."""
        ln = np.asarray(lengths, dtype=np.uint32)
        b = shard_bounds(ln, world)
        lo, hi = b[rank], b[rank + 1]
        start = np.zeros(ln.size + 1, dtype=np.uint64)
        np.cumsum(ln, dtype=np.uint64, out=start[1:])
        blo, bhi = int(start[lo]), int(start[hi])
        return RankShard(rank, world, lo, hi, blo, bhi, start[lo:hi] - np.uint64(blo), ln[lo:hi].copy())


def timed_steps(step, steps: int, sync, dist=None, max_tensor=None):
    """The timed region of the bench contract: barrier + sync, exactly `steps`
    calls of `step`, sync (this rank's own time), barrier, then the max over
    ranks.  `max_tensor(x)` wraps a float for the all-reduce (a device tensor
    under RCCL, a CPU one under gloo).  Returns (own_seconds, max_seconds)."""
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    own = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        t = max_tensor(el)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return own, el


def gather_ranks(own: dict, dist=None, world: int = 1):
    """Every rank's per-GPU record, on every rank (list indexed by rank)."""
    if dist is None:
        return [own]
    out = [None] * world
    dist.all_gather_object(out, own)
    return out


def aggregate(per_rank, steps: int, el_max: float) -> dict:
    """Whole-job figures from the gathered per-rank records (each carries
    'payload_bytes' per step): total bytes over all ranks / the max-over-ranks
    time (the contract's `value`), plus the load balance."""
    total = sum(int(r["payload_bytes"]) for r in per_rank)
    shares = [int(r["payload_bytes"]) for r in per_rank]
    return {"total_bytes_per_step": total,
            "GiB_per_s": total * steps / 2**30 / el_max if el_max > 0 else 0.0,
            "ms_per_step": el_max / steps * 1e3 if steps else 0.0,
            "imbalance": (max(shares) / (total / len(shares))) if total else 1.0}
