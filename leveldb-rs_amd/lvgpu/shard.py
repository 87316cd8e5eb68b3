"""Sharding of a batch across GPUs (one process per GPU, torch.distributed).

Buffers are independent, so a batch splits into contiguous index ranges, one
per rank, with no data-path collective.  Ranges are balanced
by payload bytes (a prefix sum of the lengths), not by count, so a Zipf mix
of 32 B records and 64 KiB blocks still loads every GPU equally.
"""
from __future__ import annotations

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
