"""Sharding of a batch across GPUs (one process per GPU, torch.distributed).

Buffers are independent, so a batch splits into contiguous index ranges, one
per rank, with no data-path collective.  Ranges are
balanced by payload bytes (a prefix sum of the lengths), not by count, so a
Zipf mix of 32 B records and 64 KiB blocks still loads every GPU equally;
fixed-size blocks (C3/C5) split by count.

The functions below are the whole N > 1 host logic of `bench.py`: the
process launcher (`launch`: `bench.py --gpus N` started without torchrun
starts its N ranks itself), the rank's range of a global batch
(`RankShard`), the timed region between barriers with the max over ranks
(`timed_steps`), and the gather of per-rank figures into the aggregate
(`gather_ranks`, `aggregate`).  The world-size-2 gloo tests
(tests/test_dist.py) drive the same functions, the launcher included, with
the CPU oracle as the per-rank compute.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from dataclasses import dataclass

import numpy as np

# torchrun's rendezvous variables; `launch` sets them for every child.
RANK_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "MASTER_ADDR", "MASTER_PORT")


def world_from_env(requested: int, env=None):
    """(world, rank, local_rank) of this process.

    Without WORLD_SIZE the process is a plain single-rank run (or the parent
    of a self-launch, see `launch`).  With WORLD_SIZE (torchrun, or a child
    of `launch`) the world must be the size the caller asked for: a bench
    told `--gpus 8` that finds itself in a world of 4 would time the wrong
    job, so that is an error, not a warning."""
    env = os.environ if env is None else env
    if "WORLD_SIZE" not in env:
        return 1, 0, 0
    world = int(env["WORLD_SIZE"])
    if world != requested:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {requested}: launch {requested} ranks "
                         f"(torchrun --nproc-per-node {requested}) or pass --gpus {world}")
    rank = int(env.get("RANK", "0"))
    local = int(env.get("LOCAL_RANK", str(rank)))
    if not (0 <= rank < world):
        raise SystemExit(f"RANK={rank} outside WORLD_SIZE={world}")
    return world, rank, local


def free_port(host: str = "127.0.0.1") -> int:
    """A port that was free a moment ago (tests that start their own groups).
    `launch` does not use it: between the probe and rank 0 binding it another
    process could take the port, so the launcher hosts the store itself."""
    s = socket.socket()
    s.bind((host, 0))
    port = s.getsockname()[1]
    s.close()
    return port


def host_store(master_addr: str = "127.0.0.1", nprocs: int = 1):
    """A TCPStore server owned by the launching process, bound to a port the OS
    picks (port 0) and kept open while the ranks run, so no other process can
    take the port between its choice and the rendezvous.  The ranks reach it
    as clients: `TORCHELASTIC_USE_AGENT_STORE=True` makes env:// rendezvous
    connect every rank, rank 0 included, instead of rank 0 hosting
    (torch/distributed/rendezvous.py `_create_c10d_store`), which is how
    torchrun's agent runs it.  Only torch.distributed's store is imported:
    nothing here touches a GPU."""
    from datetime import timedelta

    from torch.distributed import TCPStore
    return TCPStore(master_addr, 0, nprocs, is_master=True, wait_for_workers=False,
                    timeout=timedelta(seconds=900))


def launch(argv, nprocs: int, env=None, master_addr: str = "127.0.0.1", master_port: int = None,
           timeout: float = None) -> int:
    """Start `nprocs` ranks of `argv` on this node, torchrun-style, and wait.

    Child r gets RANK = LOCAL_RANK = r, WORLD_SIZE = LOCAL_WORLD_SIZE =
    nprocs, GROUP_RANK = 0 and MASTER_ADDR/MASTER_PORT (a free local port
    unless given), so `torch.distributed.init_process_group()` rendezvouses
    over env:// exactly as under `python -m torch.distributed.run`.  The
    children inherit stdout/stderr: rank 0's JSON line is the job's output.

    Unless `master_port` is given, the parent hosts the rendezvous store on
    an OS-chosen port for the life of the job (`host_store`), so the port
    cannot be taken between its choice and rank 0's bind.

    The parent never initialises a GPU (it imports torch.distributed's store,
    never the library or a device): the children are started as new
    processes, not forked from a process holding a device context, and not
    exec'd over it.  If any child
    fails the others are terminated (by their own pid, never by pattern) and
    the first non-zero exit status is returned; 0 when all succeed."""
    if nprocs < 1:
        raise ValueError("nprocs must be >= 1")
    base = dict(os.environ if env is None else env)
    for k in RANK_ENV:
        base.pop(k, None)
    store = None
    if master_port:
        port = master_port
    else:
        store = host_store(master_addr, nprocs)
        port = store.port
        base["TORCHELASTIC_USE_AGENT_STORE"] = "True"
    procs = []
    try:
        for r in range(nprocs):
            e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs),
                     LOCAL_WORLD_SIZE=str(nprocs), GROUP_RANK="0", MASTER_ADDR=master_addr,
                     MASTER_PORT=str(port), LVGPU_LAUNCHER="lvgpu.shard.launch")
            procs.append(subprocess.Popen(list(argv), env=e))
        t0 = time.monotonic()
        codes = [None] * nprocs
        while any(c is None for c in codes):
            for i, p in enumerate(procs):
                if codes[i] is None:
                    codes[i] = p.poll()
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                break
            if timeout is not None and time.monotonic() - t0 > timeout:
                bad = [124]
                break
            time.sleep(0.05)
        else:
            return 0
        for p in procs:  # one rank failed (or timed out): end the rest
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        return bad[0] if bad[0] > 0 else 128 - bad[0]  # Popen reports a signal as -N
    except BaseException:
        for p in procs:
            if p.poll() is None:
                p.kill()
        raise
    finally:
        del store  # the ranks are gone: release the port


def self_launch(script: str, args, nprocs: int) -> int:
    """`python <script> <args>` as `nprocs` ranks (see `launch`)."""
    return launch([sys.executable, os.path.abspath(script)] + list(args), nprocs)


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


@dataclass
class Timing:
    """One rank's timed region (seconds).  `own`: this rank's K steps, from
    the opening barrier + sync to its closing sync; `own_max`: the max of
    `own` over ranks -- the job's wall time (SURVEY 8e "wall time (max over
    GPUs)"), which `value` divides by; `barrier_max`: the max over ranks of
    the time to the end of the closing barrier (includes the barrier's
    latency and the ranks' skew; reported beside it)."""
    own: float
    own_max: float
    barrier_max: float


def timed_steps(step, steps: int, sync, dist=None, max_tensor=None) -> Timing:
    """The timed region of the bench contract: barrier + sync, exactly `steps`
    calls of `step`, sync (this rank's own time), barrier, then the max over
    ranks of both times in one all-reduce.  `max_tensor(list)` wraps floats
    for the all-reduce (a device tensor under RCCL, a CPU one under gloo)."""
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
    own_max = own
    if dist is not None:
        t = max_tensor([own, el])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        own_max, el = (float(x) for x in t.tolist())
    return Timing(own, own_max, el)


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
    time (the contract's `value`; bench.py passes `Timing.own_max`), plus the
    load balance."""
    total = sum(int(r["payload_bytes"]) for r in per_rank)
    shares = [int(r["payload_bytes"]) for r in per_rank]
    return {"total_bytes_per_step": total,
            "GiB_per_s": total * steps / 2**30 / el_max if el_max > 0 else 0.0,
            "ms_per_step": el_max / steps * 1e3 if steps else 0.0,
            "imbalance": (max(shares) / (total / len(shares))) if total else 1.0}
