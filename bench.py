#!/usr/bin/env python3
"""Benchmark: device-resident batched CRC32C on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c4|c5]
                    [--scaling weak|strong]

One "step" = one batch CRC32C launch over this rank's whole synthetic batch,
inputs already resident in HBM.  Default workload (N=1 headline, BASELINE.json
configs[2]): 262,144 SSTable-sized 4 KiB blocks = 1 GiB per GPU, offsets
i*4096, seed 0, splitmix64 payload generated on the device.  With N>1
every rank checksums its own batch of the same shape (weak scaling, no
data-path collective; the only collectives are the timing barrier, the
max-over-ranks of the elapsed time and the gather of per-rank records).
`--scaling strong` splits ONE global batch (c5: 16,777,216 x 4 KiB = 64 GiB,
SURVEY 8d C5 / 8e) into contiguous rank ranges instead (lvgpu.shard).

N>1 runs either under `python -m torch.distributed.run --nproc-per-node N
... bench.py --gpus N` or as plain `python bench.py --gpus N`, which starts
the N ranks itself (lvgpu.shard.launch, torchrun's environment, env://
rendezvous on 127.0.0.1) before anything touches a GPU.  A WORLD_SIZE that
differs from --gpus is an error.  Every rank's record in `per_gpu` carries
its device's PCI bus id, so N distinct devices are visible in the line.

Before the W warmup steps a `settle` phase runs back-to-back launches until
the chip's idle->busy power transient has passed (reported in the JSON line,
separate from `warmup`; see settle()).

Prints ONE JSON line on rank 0 (contract in the task statement), with
`roofline` (kernel launch duration by HIP events on the launch stream vs the
8 TB/s HBM3E peak) and `cpu_baseline` (the CPU oracle — a restatement of the
reference's SSE4.2 `extend_hw`, crc32c.rs:86-118 — timed single-threaded on
this host over a bounded sample of the same blocks).
"""
import argparse
import ctypes
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "leveldb-rs_amd"))

METRIC = "GiB/s device-resident batched CRC32C, 4KiB blocks; %HBM-peak at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md), GB/s
PAYLOAD_SEED = 0x4C444231
SETTLE = True  # --no-settle clears it (the event-timed diagnostics honour it too)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # MI355X needs ~50-60 back-to-back 1 GiB launches (~12 ms) before its
    # clocks settle (launch time drifts 0.17 -> 0.24 -> 0.17 ms); the default
    # warmup covers that transient so the timed steps are steady state.
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=100)
    p.add_argument("--workload", default="c3", choices=["c3", "c2", "c4", "c5", "kib", "tiny"],
                   help="c2-c5: SURVEY 8d configs; kib (1 M x 1 KiB) and tiny (1 M x 1-64 B): "
                        "offsets-API diagnostics for the small length classes")
    p.add_argument("--api", default="strided", choices=["offsets", "strided"],
                   help="strided = lv_crc32c_batch_strided (fixed-size table blocks); "
                        "offsets = lv_crc32c_batch_device (arbitrary buffers)")
    p.add_argument("--group", type=int, default=None, choices=[1, 4, 16, 64],
                   help="force the kernel's lanes-per-buffer group size (tuning)")
    p.add_argument("--blocks", type=int, default=None, help="override the c3/c5 block count (diagnostics)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    p.add_argument("--e2e", action="store_true",
                   help="time the host-memory path lv_crc32c_batch_host (pageable and pinned input) on C3")
    p.add_argument("--wal", action="store_true",
                   help="WAL rows of SURVEY 8f: time lv_wal_encode_host and lv_wal_scan_host (+ reader) on a "
                        "~1 GiB log of Random(301).skewed(17) records; one JSON line")
    p.add_argument("--table", action="store_true",
                   help="SURVEY 8f row 3: seal + verify SSTable block trailers of a 1 GiB table in HBM "
                        "(262,144 blocks of 4096-4351 B); one JSON line")
    p.add_argument("--hash", action="store_true",
                   help="SURVEY 8f row 4: batched hash() + cache shard of 16 M byte-packed keys (8-64 B) in HBM; "
                        "one JSON line")
    p.add_argument("--sweep", action="store_true",
                   help="north-star range: 4, 8, 16, 32, 64 KiB blocks (2 GiB per size) through the strided "
                        "(aligned) and offsets (byte-packed, 13-B misaligned) APIs; one JSON line")
    p.add_argument("--c1", action="store_true",
                   help="CPU-only config 1: the benches/crc32c.rs sweep (oracle extend_sw/extend_hw and the "
                        "product's scalar drop-ins), one JSON line; no GPU")
    p.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                   help="weak: every rank checksums its own batch of the workload's shape (default); "
                        "strong: one global batch (c5 = 64 GiB) split into contiguous rank ranges (SURVEY 8e)")
    p.add_argument("--no-settle", dest="settle", action="store_false",
                   help="skip the settle phase (back-to-back launches until the idle->busy power transient "
                        "has passed; reported as `settle`, separate from --warmup)")
    p.add_argument("--long", action="store_true",
                   help="few long buffers through both device APIs (1,024 x 64 KiB, 64 x 16 MiB, 16 x 1 MiB, "
                        "1 x 16 MiB); one JSON line")
    p.add_argument("--wal-device", action="store_true",
                   help="SURVEY 8f row 1 in HBM: lv_wal_scan_device (framing + CRC) of a ~1 GiB log already on "
                        "the GPU; one JSON line with a roofline")
    p.add_argument("--as-rank", type=int, default=0, help=argparse.SUPPRESS)
    p.add_argument("--as-world", type=int, default=1, help=argparse.SUPPRESS)
    p.add_argument("--traffic", default="auto", choices=["auto", "off"],
                   help="auto: measure roofline.traffic in a child rocprofv3 --pmc FETCH_SIZE pass")
    return p.parse_args()


def build_workload(torch, lvgpu, name, dev, rank, blocks=None):
    """Returns (arena, off, len, nbytes, description) on `dev`."""
    import numpy as np
    seed = PAYLOAD_SEED ^ (rank * 0x9E3779B9)
    if name in ("c3", "c5"):
        n = 262144 if name == "c3" else 2097152  # c5: 64 GiB over 8 GPUs = 8 GiB per GPU
        if blocks:
            n = blocks
        bl = 4096
        arena = torch.empty(n * bl, dtype=torch.uint8, device=dev)
        lvgpu.fill_splitmix(arena, 0, seed)
        off = torch.arange(n, dtype=torch.int64, device=dev) * bl
        ln = torch.full((n,), bl, dtype=torch.int32, device=dev)
        desc = f"{name}: {n} x {bl} B SSTable blocks per GPU ({n * bl / 2**30:.0f} GiB), offsets i*{bl}, seed 0"
        return arena, off, ln, n * bl, desc
    rng = np.random.default_rng(0xC0FFEE + rank)
    if name == "c4":  # Zipf(1.1) multiples of 32 B, truncated to 1..2048 (not clipped:
        # clipping rng.zipf at 2048 would pile ~44% of the mass onto 64 KiB)
        kk = np.arange(1, 2049, dtype=np.float64)
        cdf = np.cumsum(kk ** -1.1)
        cdf /= cdf[-1]
        k = np.searchsorted(cdf, rng.random(1048576), side="right") + 1
        k = np.minimum(k, 2048)
        lens = (32 * k).astype(np.uint32)
        desc = "c4: 1,048,576 buffers, L = 32*k, k ~ Zipf(1.1) on 1..2048, byte-packed"
    elif name in ("kib", "tiny"):
        lens = (np.full(1048576, 1024) if name == "kib" else rng.integers(1, 65, 1048576)).astype(np.uint32)
        desc = f"{name}: 1,048,576 buffers of " + ("1 KiB" if name == "kib" else "1-64 B") + ", byte-packed"
    else:  # c2: WAL physical records from Random(301).skewed(17) record sizes
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        lens = wal_unit_lengths(1048576)
        desc = "c2: 1,048,576 WAL CRC units [type||fragment], sizes from Random(301).skewed(17) fragmented per add_record"
    offs = np.zeros(lens.size, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    total = int(offs[-1] + lens[-1])
    arena = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(arena, 0, seed)
    off = torch.from_numpy(offs.astype(np.int64)).to(dev)
    ln = torch.from_numpy(lens.view(np.int32)).to(dev)
    return arena, off, ln, total, desc


def wal_unit_lengths(n):
    """CRC unit lengths (1 + fragment) of the WAL the reference writer produces for
    records of size Random(301).skewed(17) (log_writer.rs:62-110, random.rs:66-69)."""
    import numpy as np
    B, H = 32768, 7
    out = np.empty(n, dtype=np.uint32)
    m = 0
    state = 301 & 0x7FFFFFFF
    block_off = 0

    def nxt():
        nonlocal state
        prod = state * 16807
        s = ((prod >> 31) + (prod & 2147483647)) & 0xFFFFFFFF
        if s > 2147483647:
            s -= 2147483647
        state = s
        return s
    while m < n:
        r = 1 << (nxt() % 18)
        left = nxt() % r
        while m < n:
            if B - block_off < H:
                block_off = 0
            avail = B - block_off - H
            frag = min(left, avail)
            out[m] = frag + 1
            m += 1
            block_off += H + frag
            left -= frag
            if left <= 0:
                break
    return out


def read_pmc_traffic(path):
    """HBM bytes per step from a rocprofv3 --pmc CSV.  A step is one launch of
    each lvk:: kernel the call makes (the blocks kernel for the strided API;
    the three sort kernels + the persistent class kernel for the
    offsets API), so the per-step figure is the sum over kernel names of each
    name's mean FETCH_SIZE (the fill kernel excluded).  FETCH_SIZE is in KiB
    and, on gfx950, counts half the bytes of a wide 16-B-per-lane streaming
    read, so it is doubled (MI355X_MICROARCH.md §HBM)."""
    import collections
    import csv
    per = collections.defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            if "lvk::" in name and "fill_" not in name and row.get("Counter_Name") == "FETCH_SIZE":
                per[name].append(float(row["Counter_Value"]))
    if not per:
        return None
    return 2.0 * 1024.0 * sum(sum(v) / len(v) for v in per.values())


def measure_traffic(args, shard_rank=0, shard_world=1):
    """Child process: rocprofv3 --pmc FETCH_SIZE over a short run of the same
    workload (a separate pass, kernel counters only).  Returns bytes/launch.
    In an N-rank job rank 0 runs it after the timed region, as a single
    process replaying its own shard (--as-rank/--as-world; the torchrun
    variables are dropped so the child does not join the process group)."""
    import glob
    import shutil
    import subprocess
    import tempfile
    from lvgpu import shard
    exe = shutil.which("rocprofv3")
    if exe is None:
        return None, "rocprofv3 not found"
    if any(k.startswith("ROCPROF") for k in os.environ):  # already under a profiler: never nest one
        return None, "skipped (running under rocprofv3)"
    out = tempfile.mkdtemp(prefix="lvgpu_pmc_", dir="/tmp")
    cmd = [exe, "--pmc", "FETCH_SIZE", "--output-format", "csv", "-d", out, "-o", "pmc", "--",
           sys.executable, os.path.abspath(__file__), "--steps", "10", "--warmup", "60", "--cpu-seconds", "0",
           "--traffic", "off", "--no-settle", "--workload", args.workload, "--api", args.api,
           "--scaling", args.scaling,  # bytes per launch do not depend on the clock state: no settle
           "--as-rank", str(shard_rank), "--as-world", str(shard_world)]
    if args.group:
        cmd += ["--group", str(args.group)]
    if args.blocks:
        cmd += ["--blocks", str(args.blocks)]
    env = {k: v for k, v in os.environ.items() if k not in shard.RANK_ENV and k != "LVGPU_LAUNCHER"}
    env["TMPDIR"] = "/tmp"
    try:
        subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                       timeout=300, check=True)
    except Exception as e:  # noqa: BLE001 - report, never fail the bench on the profiler
        return None, f"rocprofv3 pass failed: {e}"
    files = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)
    t = read_pmc_traffic(files[0]) if files else None
    shutil.rmtree(out, ignore_errors=True)
    return t, "rocprofv3 --pmc FETCH_SIZE (x2 gfx950 correction), per step: sum over the call's kernels of each kernel's mean"


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(torch, arena, off, ln, seconds, sample_bytes=64 << 20):
    """The oracle's extend() (crc32c.rs:42-51: the SSE4.2 crc32 path of
    :86-118 on this host) over a bounded sample of the same workload: its first
    buffers up to `sample_bytes`, gathered from HBM into one packed host arena.
    One C call per pass (oracle_batch loops in C).  The reference-faithful
    figure is 1 thread (libtest's bench is single-threaded); an aggregate over
    the box's CPU share (16 threads: one Python thread per slice, ctypes drops
    the GIL) is reported beside it for context.  Returns (baseline, sample
    CRCs, sample count) so the caller can check the GPU results."""
    import threading

    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import wal_oracle as W
    L = W.lib()
    lens = ln[: 1 << 20].to(torch.int64)
    cum = torch.cumsum(lens, 0)
    k = max(1, int(torch.searchsorted(cum, torch.tensor([sample_bytes], device=cum.device)).item()))
    k = min(k, ln.numel())
    l_k = lens[:k]
    total = int(l_k.sum().item())
    starts = torch.cumsum(l_k, 0) - l_k
    # byte j of the packed sample = arena[off[b] + (j - starts[b])], b = buffer of j
    owner = torch.repeat_interleave(torch.arange(k, device=arena.device), l_k)
    idx = off[:k].to(torch.int64)[owner] + (torch.arange(total, device=arena.device) - starts[owner])
    host = np.ascontiguousarray(arena[idx].cpu().numpy()) if total else np.zeros(1, np.uint8)
    del owner, idx
    h_off = np.ascontiguousarray(starts.cpu().numpy().astype(np.uint64))
    h_len = np.ascontiguousarray(l_k.cpu().numpy().astype(np.uint32))
    crcs = np.zeros(k, dtype=np.uint32)

    def run(lo, hi, secs, out):
        passes, t0 = 0, time.perf_counter()
        while True:
            L.oracle_batch(host.ctypes.data, h_off[lo:].ctypes.data, h_len[lo:].ctypes.data, None,
                           crcs[lo:].ctypes.data, hi - lo, 0)
            passes += 1
            el = time.perf_counter() - t0
            if el >= secs:
                break
        out.append((passes * int(h_len[lo:hi].sum(dtype=np.uint64)), el))

    single = []
    run(0, k, seconds, single)
    threads = 16
    bounds = [k * t // threads for t in range(threads + 1)]
    agg, th = [], []
    for t in range(threads):
        if bounds[t + 1] > bounds[t]:
            th.append(threading.Thread(target=run, args=(bounds[t], bounds[t + 1], max(1.0, seconds / 4), agg)))
    for t in th:
        t.start()
    for t in th:
        t.join()
    agg_rate = sum(b / e for b, e in agg) / 2**30
    b1, e1 = single[0]
    return {"value": round(b1 / 2**30 / e1, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"first {k} buffers of the workload ({total / 2**20:.1f} MiB, gathered from HBM), "
                      f"{b1 // max(total, 1)} passes in {e1:.1f} s; oracle extend() = SSE4.2 crc32 path of "
                      f"crc32c.rs:86-118, 1 thread",
            "all_cores": {"value": round(agg_rate, 2), "unit": "GiB/s", "threads": len(th),
                          "note": "same sample split over the box's 16-thread CPU share, for context"},
            "host_cpu": _cpu_model(), "host_nproc": os.cpu_count()}, crcs, k


def e2e(args):
    """End-to-end rate of the host-memory path (the reference's data lives in
    host file buffers): H2D of the 1 GiB C3 arena + kernel + D2H of the CRCs,
    synchronous per call.  Pageable input goes through the pipelined pinned
    staging; pinned input is DMA'd directly."""
    import numpy as np
    import torch
    import lvgpu
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import wal_oracle as W
    n, bl = (args.blocks or 262144), 4096
    host = np.empty(n * bl, dtype=np.uint8)
    W.lib().oracle_fill_splitmix(host.ctypes.data, 0, host.size, PAYLOAD_SEED)
    off = np.arange(n, dtype=np.uint64) * bl
    ln = np.full(n, bl, dtype=np.uint32)
    pinned = torch.empty(host.size, dtype=torch.uint8, pin_memory=True)
    pinned.numpy()[:] = host
    res = {}
    for name, arr in (("pageable", host), ("pinned", pinned.numpy())):
        lvgpu.batch_host(arr, off, ln)  # warm: allocations, staging
        ts = []
        for _ in range(max(3, args.steps // 20)):
            t0 = time.perf_counter()
            out = lvgpu.batch_host(arr, off, ln)
            ts.append(time.perf_counter() - t0)
        ts.sort()
        med = ts[len(ts) // 2]
        res[name] = {"GiB_per_s": round(n * bl / 2**30 / med, 2), "ms": round(med * 1e3, 2)}
        want = np.zeros(1024, dtype=np.uint32)
        W.lib().oracle_batch(host.ctypes.data, off.ctypes.data, ln.ctypes.data, None, want.ctypes.data, 1024, 0)
        assert (out[:1024] == want).all(), "e2e parity check failed"
    print(json.dumps({"metric": "end-to-end host-memory batched CRC32C (H2D + kernel + D2H), C3 1 GiB",
                      "unit": "GiB/s", "results": res, "blocks": n, "block_bytes": bl}), flush=True)


def c1_sweep(args):
    """BASELINE configs[0] / SURVEY 8d C1: benches/crc32c.rs restated — one
    thread, a vec!['x'; N] buffer, extend_sw(0, .) and extend_hw(0, .) per
    iteration (benches/crc32c.rs:23-61), sizes {256, 4096, 60056, 1 Mi, 16 Mi}
    plus the 1-64 KiB sweep; median of 5 runs of ~0.2 s per size and path.
    The oracle is the reference restatement; lv_crc32c_extend_{sw,hw} are the
    product's host scalar drop-ins (same answers, timed for comparison)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import lvgpu
    import wal_oracle as W
    O, P = W.lib(), lvgpu.lib()
    sizes = sorted({256, 4096, 60056, 1 << 20, 16 << 20} | {k << 10 for k in (1, 2, 4, 8, 16, 32, 64)})

    def rate(fn, n):
        iters = 1
        while True:  # calibrate to ~0.2 s per run
            t0 = time.perf_counter()
            fn(iters)
            el = time.perf_counter() - t0
            if el > 0.05:
                break
            iters *= 4
        iters = max(1, int(iters * 0.2 / el))
        runs = []
        for _ in range(5):
            t0 = time.perf_counter()
            fn(iters)
            runs.append(time.perf_counter() - t0)
        runs.sort()
        return round(n * iters / runs[2] / 2**30, 3)

    rows = []
    for n in sizes:
        buf = (ctypes.c_uint8 * n).from_buffer(bytearray(b"x" * n))
        b = bytes(buf)
        assert O.oracle_extend_hw(0, b, n) == P.lv_crc32c_extend_hw(0, b, n) == P.lv_crc32c_extend_sw(0, b, n)
        row = {"bytes": n,
               "ref_sw": rate(lambda it: O.oracle_bench_loop(buf, n, it, 0), n),
               "ref_hw": rate(lambda it: O.oracle_bench_loop(buf, n, it, 1), n)}

        def loop(fn, it):
            for _ in range(it):
                fn(0, b, n)
        row["lvgpu_sw"] = rate(lambda it: loop(P.lv_crc32c_extend_sw, it), n) if n >= 4096 else None
        row["lvgpu_hw"] = rate(lambda it: loop(P.lv_crc32c_extend_hw, it), n) if n >= 4096 else None
        rows.append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    print(json.dumps({"metric": "benches/crc32c.rs CPU sweep (config 1), GiB/s single thread", "unit": "GiB/s",
                      "host_cpu": _cpu_model(), "host_nproc": os.cpu_count(),
                      "note": "ref_* = oracle restatement in one C loop; lvgpu_* = product scalar via ctypes "
                              "(per-call overhead included, so only sizes >= 4 KiB are reported)",
                      "results": rows}), flush=True)


def _event_times(torch, fn, steps, warmup):
    """Median and mean ms of `fn` by HIP events on the current stream, after
    the settle phase (see settle()) and `warmup` calls."""
    if SETTLE:
        settle(torch, fn, torch.cuda.current_stream())
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in evs)
    return ts[len(ts) // 2], sum(ts) / len(ts)


def sweep_bench(args):
    """BASELINE.json's target range, '>= 70 % of HBM peak on 4-64 KiB blocks':
    per block size, 2 GiB of blocks in HBM, (a) lv_crc32c_batch_strided on
    aligned blocks (uniform-block kernel) and (b) lv_crc32c_batch_device on
    the same sizes byte-packed from a 13-B offset (every block misaligned:
    sort + class kernel).  HIP-event mean over the timed launches; 64 blocks
    of each configuration are checked against the oracle in the run."""
    import numpy as np
    import torch
    import lvgpu
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import wal_oracle as W
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    lvgpu.device_init()
    total = 2 << 30
    arena = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(arena, 0, PAYLOAD_SEED)
    L = W.lib()
    rows = []
    steps, warm = max(20, min(args.steps, 100)), max(20, min(args.warmup, 60))
    for kib in (4, 8, 16, 32, 64):
        bl = kib << 10
        n = total // bl
        out = torch.empty(n, dtype=torch.int32, device=dev)
        offs = np.arange(n, dtype=np.int64) * bl + 13
        o = torch.from_numpy(offs).to(dev)
        ln = torch.full((n,), bl, dtype=torch.int32, device=dev)
        ws = torch.empty(lvgpu.workspace_bytes(n), dtype=torch.uint8, device=dev)
        row = {"block_KiB": kib, "blocks": n}
        for api, fn in (("strided", lambda: lvgpu.batch_strided(arena, bl, bl, n, out=out)),
                        ("offsets", lambda: lvgpu.batch_ws(arena, o, ln, ws, out=out))):
            _, avg = _event_times(torch, fn, steps, warm)
            fn()
            torch.cuda.synchronize()
            k = 64
            base = 0 if api == "strided" else 13
            host = arena[:base + k * bl].cpu().numpy()
            want = np.zeros(k, dtype=np.uint32)
            ho = (np.arange(k, dtype=np.uint64) * bl + base).astype(np.uint64)
            hl = np.full(k, bl, dtype=np.uint32)
            L.oracle_batch(host.ctypes.data, ho.ctypes.data, hl.ctypes.data, None, want.ctypes.data, k, 0)
            if not np.array_equal(out[:k].cpu().numpy().view(np.uint32), want):
                raise SystemExit(f"sweep parity check failed ({api}, {kib} KiB)")
            gbs = n * bl / (avg * 1e-3) / 1e9
            row[api] = {"GB_per_s": round(gbs, 1), "frac_of_8TBps": round(gbs / HBM_PEAK_GBS, 4),
                        "ms_avg": round(avg, 4)}
        rows.append(row)
        del out, o, ln, ws
    res = {"metric": "device-resident batched CRC32C across the 4-64 KiB target range", "unit": "GB/s",
           "bytes_per_size": total, "results": rows,
           "timing": "HIP events around each call, mean of the timed launches after warmup",
           "data": "synthetic splitmix64 payload in HBM"}
    print(json.dumps(res), flush=True)
    return res


def long_bench(args):
    """Few long buffers (verdict r01: intra-buffer parallelism; the reference
    bench's 1 MiB / 16 MiB buffers, benches/crc32c.rs:59-60): 1,024 x 64 KiB,
    64 x 16 MiB, 16 x 1 MiB and 1 x 16 MiB blocks in HBM through the strided
    API (long-block split + device-side combine) and the offsets API.
    HIP-event mean per call (all kernels of the call); 4 buffers of each
    configuration checked against the oracle in the run."""
    import numpy as np
    import torch
    import lvgpu
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import wal_oracle as W
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    lvgpu.device_init()
    L = W.lib()
    rows = []
    for n, bl in ((1024, 64 << 10), (64, 16 << 20), (16, 1 << 20), (1, 16 << 20)):
        arena = torch.empty(n * bl + 64, dtype=torch.uint8, device=dev)
        lvgpu.fill_splitmix(arena, 0, PAYLOAD_SEED)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        o = torch.arange(n, dtype=torch.int64, device=dev) * bl
        ln = torch.full((n,), bl, dtype=torch.int32, device=dev)
        ws = torch.empty(lvgpu.workspace_bytes(n), dtype=torch.uint8, device=dev)
        row = {"blocks": n, "block_bytes": bl}
        for api, fn in (("strided", lambda: lvgpu.batch_strided(arena, bl, bl, n, out=out)),
                        ("offsets", lambda: lvgpu.batch_ws(arena, o, ln, ws, out=out))):
            p50, avg = _event_times(torch, fn, max(20, min(args.steps, 100)), max(10, min(args.warmup, 50)))
            fn()
            kern = lvgpu.last_kernel()
            torch.cuda.synchronize()
            k = min(n, 4)
            host = arena[:k * bl].cpu().numpy()
            want = np.zeros(k, dtype=np.uint32)
            ho = np.arange(k, dtype=np.uint64) * bl
            hl = np.full(k, bl, dtype=np.uint32)
            L.oracle_batch(host.ctypes.data, ho.ctypes.data, hl.ctypes.data, None, want.ctypes.data, k, 0)
            if not np.array_equal(out[:k].cpu().numpy().view(np.uint32), want):
                raise SystemExit(f"long-buffer parity check failed ({api}, {n} x {bl})")
            gbs = n * bl / (avg * 1e-3) / 1e9
            row[api] = {"GB_per_s": round(gbs, 1), "frac_of_8TBps": round(gbs / HBM_PEAK_GBS, 4),
                        "us_avg": round(avg * 1e3, 2), "us_p50": round(p50 * 1e3, 2), "kernels": kern}
        rows.append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
        del arena, out, o, ln, ws
    res = {"metric": "few long buffers, device-resident batched CRC32C", "unit": "GB/s", "results": rows,
           "timing": "HIP events around each call (every kernel of the call), mean (us_avg) and median "
                     "(us_p50) after settle + warmup; a ~20 us call's mean carries the odd slow call",
           "data": "synthetic splitmix64 payload in HBM"}
    print(json.dumps(res), flush=True)
    return res


def wal_device_bench(args):
    """SURVEY 8f row 1 in HBM (verdict r01 "missing" 3): lv_wal_scan_device
    over a ~1 GiB log of Random(301).skewed(17) records already on the GPU:
    each 32 KiB block's header chain is walked inside the length sort's passes
    (wal_hist, wal_scatter), every [type || payload] unit is checksummed by the
    class kernel, records land in log order -- four launches, no host sync.
    (A fused one-pass scan measured slower: profiles/r02/walfused/.)
    Algorithmic bytes: the log (every byte read once by the CRC; the framing
    reads the 7-B headers again).  HIP-event mean per call; the whole scan is
    checked against the oracle's framing (first 2000 records' CRCs vs value())."""
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import lvgpu
    import lvgpu.wal as LW
    import wal_oracle as W
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    lvgpu.device_init()
    target = (args.blocks or 262144) * 4096
    r = W.Random(301)
    sizes, tot = [], 0
    while tot < target:
        n = r.skewed(17)
        sizes.append(n)
        tot += n
    sizes = np.array(sizes, dtype=np.uint64)
    rng = np.random.default_rng(7)
    payload = rng.integers(0, 256, size=int(tot), dtype=np.uint8)
    offs = np.zeros(sizes.size, dtype=np.uint64)
    offs[1:] = np.cumsum(sizes[:-1])
    L = LW._bind()
    need = ctypes.c_size_t()
    L.lv_wal_encode_host(payload.ctypes.data, offs.ctypes.data, sizes.ctypes.data, sizes.size, 0, None, 0,
                         ctypes.byref(need), 0)
    log = np.empty(need.value, dtype=np.uint8)
    if L.lv_wal_encode_host(payload.ctypes.data, offs.ctypes.data, sizes.ctypes.data, sizes.size, 0,
                            log.ctypes.data, log.size, ctypes.byref(need), 0):
        raise SystemExit("encode failed: " + lvgpu.lib().lv_last_error().decode())
    del payload
    d_log = torch.from_numpy(log).to(dev)
    # capacity from a first scan (a caller learns its log's record count once)
    _, _, _, count = LW.scan_device(d_log, 0)
    torch.cuda.synchronize()
    cap = int(count.item())
    ws = torch.empty(LW.scan_workspace_bytes(log.size, cap), dtype=torch.uint8, device=dev)
    hdr = torch.empty(cap, dtype=torch.int64, device=dev)
    crc = torch.empty(cap, dtype=torch.int32, device=dev)
    info = torch.empty(cap, dtype=torch.int32, device=dev)
    cnt = torch.empty(1, dtype=torch.int64, device=dev)
    from lvgpu import _dev_ptr, _stream_ptr

    def scan():
        rc = L.lv_wal_scan_device(_dev_ptr(d_log, "log"), log.size, _dev_ptr(hdr, "h"), _dev_ptr(crc, "c"),
                                  _dev_ptr(info, "i"), cap, _dev_ptr(cnt, "n"), _dev_ptr(ws, "ws"), ws.numel(),
                                  _stream_ptr(None))
        if rc:
            raise SystemExit("lv_wal_scan_device failed: " + lvgpu.lib().lv_last_error().decode())
    p50, avg = _event_times(torch, scan, max(20, min(args.steps, 100)), max(10, min(args.warmup, 50)))
    scan()
    torch.cuda.synchronize()
    assert int(cnt.item()) == cap
    o, c, i = W.scan_log(log.tobytes()) if log.size <= (256 << 20) else (None, None, None)
    parity = ""
    h_hdr, h_crc, h_info = hdr.cpu().numpy(), crc.cpu().numpy().view(np.uint32), info.cpu().numpy().view(np.uint32)
    if os.environ.get("LVGPU_EXPERIMENT") == "1":  # timing variants compute wrong CRCs
        o = None
        parity = "none (experiment variant)"
    elif o is not None:
        if not (h_hdr.tolist() == o and h_crc.tolist() == c and h_info.tolist() == i):
            raise SystemExit("WAL device scan differs from the oracle framing")
        parity = "whole scan == oracle.scan_log"
    elif parity != "none (experiment variant)":
        raw = log.tobytes()
        for k in range(min(2000, cap)):
            ln = int(h_info[k]) >> 16
            st = (int(h_info[k]) >> 8) & 0xff
            if st == 0 and int(h_crc[k]) != W.value(raw[int(h_hdr[k]) + 6:int(h_hdr[k]) + 7 + ln]):
                raise SystemExit("WAL device scan parity check failed")
        parity = "first 2000 records' CRCs vs oracle value()"
    gbs = log.size / (avg * 1e-3) / 1e9
    res = {"metric": "device-resident WAL verify scan (framing + CRC of every record), HBM", "unit": "GB/s",
           "log_bytes": int(log.size), "records": int(sizes.size), "physical_records": cap,
           "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(gbs / HBM_PEAK_GBS, 4), "ms_avg": round(avg, 4), "ms_p50": round(p50, 4),
                        "bytes_per_call": int(log.size),
                        "kernels": lvgpu.last_kernel()},
           "api": "lv_wal_scan_device", "parity": parity,
           "timing": "HIP events around each call (all of its kernels), mean after settle + warmup",
           "data": "synthetic: Random(301).skewed(17) record sizes, random payload, encoded by lv_wal_encode_host"}
    print(json.dumps(res), flush=True)
    return res


def table_bench(args):
    """SURVEY 8f row 3 in HBM: lv_sst_seal_blocks_device writes the
    type(1) || mask(crc32c(contents || type)) trailer of every block of a table
    being built; lv_sst_verify_blocks_device checks them (table/format.rs
    BlockHandle extents; trailer layout parity unpinned).  Blocks of
    4096 + U[0, 256) bytes (a 4 KiB block_size threshold overshoots by up to
    one entry), each followed by its 5-byte trailer; ~1 GiB.  Algorithmic
    bytes: contents + type (seal also writes 4 B, verify reads 4 B)."""
    import numpy as np
    import torch
    import lvgpu
    import lvgpu.table as T
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import wal_oracle as W
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    lvgpu.device_init()
    n = args.blocks or 262144
    rng = np.random.default_rng(0x55AB1E)
    sizes = (4096 + rng.integers(0, 256, n)).astype(np.int64)
    offs = np.zeros(n, dtype=np.int64)
    offs[1:] = np.cumsum(sizes[:-1] + 5)
    total = int(offs[-1] + sizes[-1] + 5)
    f = torch.empty(total, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(f, 0, PAYLOAD_SEED)
    h = torch.from_numpy(np.stack([offs, sizes], axis=1).copy()).to(dev)
    seal_p50, seal_avg = _event_times(torch, lambda: T.seal_blocks(f, h), args.steps, args.warmup)
    ver_p50, ver_avg = _event_times(torch, lambda: T.verify_blocks(f, h), args.steps, args.warmup)
    st, crc = T.verify_blocks(f, h, out_crc=True)
    torch.cuda.synchronize()
    # timing studies of experiment variants (wrong CRCs by design) skip parity
    variant = lvgpu.experiment_variant()
    if not variant and not bool((st == T.BLOCK_OK).all()):
        raise SystemExit("table bench: a sealed block failed verification")
    host = f[:int(offs[min(n, 2000) - 1] + sizes[min(n, 2000) - 1] + 1)].cpu().numpy().tobytes()
    got = crc[:2000].cpu().numpy().view(np.uint32)
    for k in range(0 if variant else min(n, 2000)):
        o, sz = int(offs[k]), int(sizes[k])
        if W.value(host[o:o + sz + 1]) != int(got[k]):
            raise SystemExit("table bench parity check failed")
    unit = int(sizes.sum()) + n  # contents + type byte per block
    res = {"metric": "SSTable block trailer seal / verify, device-resident", "unit": "GiB/s",
           "blocks": n, "bytes_per_call": unit, "table_bytes": total,
           "seal": {"GiB_per_s": round(unit / 2**30 / (seal_avg * 1e-3), 1), "ms_avg": round(seal_avg, 4),
                    "ms_p50": round(seal_p50, 4), "frac_of_8TBps": round(unit / (seal_avg * 1e-3) / 8e12, 4)},
           "verify": {"GiB_per_s": round(unit / 2**30 / (ver_avg * 1e-3), 1), "ms_avg": round(ver_avg, 4),
                      "ms_p50": round(ver_p50, 4), "frac_of_8TBps": round(unit / (ver_avg * 1e-3) / 8e12, 4)},
           "timing": "HIP events around each call (CRC batch + trailer kernels)", "parity": "first 2000 blocks vs oracle",
           "data": "synthetic splitmix64 contents in HBM"}
    print(json.dumps(res), flush=True)
    return res


def hash_bench(args):
    """SURVEY 8f row 4 in HBM: lv_hash_batch_device over 16,777,216 byte-packed
    keys of 8-64 bytes (cache-key sized; util/hash.rs:20-51, cache shard
    cache.rs:394-399).  One lane per key (the hash is a serial chain), so the
    bound is HBM: key bytes + 12 B metadata + 4 B output per key."""
    import numpy as np
    import torch
    import lvgpu
    from lvgpu import hash as H
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import wal_oracle as W
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    lvgpu.device_init()
    n = args.blocks or 16777216
    rng = np.random.default_rng(0x4A54)
    lens = rng.integers(8, 65, n).astype(np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    total = int(offs[-1] + lens[-1])
    arena = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(arena, 0, PAYLOAD_SEED)
    o = torch.from_numpy(offs.astype(np.int64)).to(dev)
    ln = torch.from_numpy(lens.view(np.int32)).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    p50, avg = _event_times(torch, lambda: H.hash_batch(arena, o, ln, out=out, shard=True), args.steps, args.warmup)
    H.hash_batch(arena, o, ln, out=out)
    torch.cuda.synchronize()
    L = W.lib()
    L.oracle_hash_batch.restype = None
    L.oracle_hash_batch.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t]
    k = min(n, 100000)
    host = arena[:int(offs[k - 1] + lens[k - 1])].cpu().numpy()
    want = np.zeros(k, dtype=np.uint32)
    L.oracle_hash_batch(host.ctypes.data, offs[:k].ctypes.data, lens[:k].ctypes.data, None, want.ctypes.data, k)
    if not np.array_equal(out[:k].cpu().numpy().view(np.uint32), want):
        raise SystemExit("hash bench parity check failed")
    moved = total + 16 * n  # key bytes + off/len + out
    res = {"metric": "batched leveldb hash() + cache shard, device-resident", "unit": "Gkeys/s",
           "keys": n, "key_bytes": total, "value": round(n / (avg * 1e-3) / 1e9, 3), "ms_avg": round(avg, 4),
           "ms_p50": round(p50, 4), "hbm_GB_per_s": round(moved / (avg * 1e-3) / 1e9, 1),
           "frac_of_8TBps": round(moved / (avg * 1e-3) / 8e12, 4),
           "note": "hbm bytes = key bytes + 8 B offset + 4 B length + 4 B output per key",
           "parity": "first 100000 keys vs oracle", "data": "synthetic splitmix64 keys in HBM"}
    print(json.dumps(res), flush=True)
    return res


def wal_bench(args):
    """SURVEY 8f rows 1-2 end to end from host memory: group-commit encode
    (lv_wal_encode_host: layout + one GPU CRC batch) and whole-log verify
    (lv_wal_scan_host: H2D, block framing, one CRC batch, D2H), then the host
    Reader over the scan.  Records: logical sizes Random(301).skewed(17)
    (log_writer.rs:456-458, 567), random payload, until ~1 GiB.  The first
    2000 physical records' CRCs are checked against the oracle."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import lvgpu
    import lvgpu.wal as LW
    import wal_oracle as W
    target = (args.blocks or 262144) * 4096
    r = W.Random(301)
    sizes = []
    tot = 0
    while tot < target:
        n = r.skewed(17)
        sizes.append(n)
        tot += n
    sizes = np.array(sizes, dtype=np.uint64)
    rng = np.random.default_rng(7)
    payload = rng.integers(0, 256, size=int(tot), dtype=np.uint8)
    offs = np.zeros(sizes.size, dtype=np.uint64)
    offs[1:] = np.cumsum(sizes[:-1])
    L = LW._bind()
    need = ctypes.c_size_t()
    L.lv_wal_encode_host(payload.ctypes.data, offs.ctypes.data, sizes.ctypes.data, sizes.size, 0, None, 0,
                         ctypes.byref(need), 0)
    out = np.empty(need.value, dtype=np.uint8)

    def encode():
        rc = L.lv_wal_encode_host(payload.ctypes.data, offs.ctypes.data, sizes.ctypes.data, sizes.size, 0,
                                  out.ctypes.data, out.size, ctypes.byref(need), 0)
        if rc:
            raise SystemExit("encode failed: " + lvgpu.lib().lv_last_error().decode())

    def scan():
        h = L.lv_wal_scan_host(out.ctypes.data, out.size, 0)
        if not h:
            raise SystemExit("scan failed: " + lvgpu.lib().lv_last_error().decode())
        return LW.Scan(h)

    def med(fn, reps):
        fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return sorted(ts)[len(ts) // 2]
    reps = max(3, min(args.steps, 10))
    t_enc = med(encode, reps)
    t_scan = med(scan, reps)
    sc = scan()
    o, c, info = sc.offsets, sc.crcs, sc.info
    log = out.tobytes()
    for k in range(min(2000, o.size)):
        ln = int(info[k]) >> 16
        assert int(c[k]) == W.value(log[int(o[k]) + 6:int(o[k]) + 7 + ln]), "scan parity check failed"
    t0 = time.perf_counter()
    rd = LW.Reader(log, sc, W.ReportCollector())
    nrec = 0
    while rd.read_record() is not None:
        nrec += 1
    t_read = time.perf_counter() - t0
    assert nrec == sizes.size, (nrec, sizes.size)
    gib = out.size / 2**30
    print(json.dumps({"metric": "WAL group-commit encode and whole-log verify, host memory end to end",
                      "unit": "GiB/s of log", "log_bytes": int(out.size), "records": int(sizes.size),
                      "physical_records": int(o.size),
                      "encode": {"GiB_per_s": round(gib / t_enc, 2), "ms": round(t_enc * 1e3, 2),
                                 "api": "lv_wal_encode_host"},
                      "scan": {"GiB_per_s": round(gib / t_scan, 2), "ms": round(t_scan * 1e3, 2),
                               "api": "lv_wal_scan_host (H2D + framing + CRC batch + D2H)"},
                      "reader_ms": round(t_read * 1e3, 1),
                      "reader_note": "host Reader replay via ctypes, one call per record (not a GPU figure)",
                      "data": "synthetic: Random(301).skewed(17) record sizes, random payload"}), flush=True)


def settle(torch, step, stream, min_s=0.6, max_s=3.0, chunk=20, window=8, tol=0.006, best_tol=0.008):
    """Run back-to-back launches until the launch time has stopped moving.

    An MI355X coming out of idle runs its first ~100 back-to-back 1 GiB
    launches through a power-management transient: launch time rises from
    0.167 to ~0.21 ms around launches 10-40 and relaxes back to 0.164 over the
    next ~100 (tools/ramp_probe.py, profiles/r02/ramp/).  It recurs after 1 s
    or 3 s of idle on the same arena and does not appear on a freshly
    allocated arena while the chip is busy, so it is the chip's idle -> busy
    clock/power state, not first touch of the memory (sysfs mclk/fclk read
    2000/1250 MHz throughout; sclk DPM does not track it).  The settle phase
    is kept apart from `warmup` so `steps`/`warmup` stay what the caller
    asked for: chunks of `chunk` launches are timed by events (two chunks in
    flight, so the queue never drains) until at least `min_s` has passed, the
    last `window` chunk times lie within `tol` of each other and their mean
    within `best_tol` of the fastest chunk so far (a slow tail of the
    transient, still improving by < 1.5 % per window, passed the round-2
    first rule of 0.3 s / 5 chunks / 1.5 % at 0.167 vs a steady 0.164 ms and
    put `frac` at 0.79 on one box), or `max_s`."""
    t0 = time.perf_counter()
    pend, times = [], []
    launches = 0
    while True:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(chunk):
            step()
        b.record(stream)
        launches += chunk
        pend.append((a, b))
        if len(pend) < 2:
            continue
        a0, b0 = pend.pop(0)
        b0.synchronize()
        times.append(a0.elapsed_time(b0) / chunk)
        el = time.perf_counter() - t0
        w = times[-window:]
        if el >= max_s or (el >= min_s and len(w) == window and max(w) <= min(w) * (1 + tol)
                           and sum(w) / window <= min(times) * (1 + best_tol)):
            break
    torch.cuda.synchronize()
    return {"launches": launches, "seconds": round(time.perf_counter() - t0, 3),
            "first_chunk_ms": round(times[0], 4), "peak_chunk_ms": round(max(times), 4),
            "last_chunk_ms": round(times[-1], 4),
            "rule": f">= {min_s} s of back-to-back launches, the last {window} chunks of {chunk} "
                    f"within {tol * 100:.1f} % and their mean within {best_tol * 100:.1f} % of the fastest "
                    f"chunk (cap {max_s} s)",
            "why": "idle->busy power transient of the chip (tools/ramp_probe.py); not part of warmup"}


class _stdout_to_stderr:
    """Points file descriptor 1 at stderr for the duration (C/C++ libraries
    write to the descriptor, not to sys.stdout)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def build_shard(torch, lvgpu, args, dev, rank, world):
    """Strong scaling: ONE global batch, this rank's
    contiguous slice of it.  c5: 16,777,216 x 4 KiB = 64 GiB; c3: 262,144 x
    4 KiB; c2/c4: the global length list split by payload bytes.  The rank
    generates only its slice's bytes of the global splitmix arena (the fill
    is indexed by global byte), so every rank reads exactly what a single GPU
    would.  Returns (arena, off, len, shard, description)."""
    from lvgpu.shard import RankShard
    import numpy as np
    if args.workload in ("c3", "c5"):
        n_total = args.blocks or (262144 if args.workload == "c3" else 16777216)
        sh = RankShard.uniform(n_total, 4096, rank, world)
        desc = (f"{args.workload}: global batch {n_total} x 4096 B ({n_total * 4096 / 2**30:.0f} GiB), "
                f"rank {rank} owns blocks [{sh.lo}, {sh.hi})")
        pad = 0
    else:
        lens = global_lengths(args.workload)
        sh = RankShard.packed(lens, rank, world)
        desc = (f"{args.workload}: global batch of {lens.size} buffers split by payload bytes, "
                f"rank {rank} owns [{sh.lo}, {sh.hi})")
        pad = 16
    arena = torch.empty(sh.byte_hi - sh.byte_lo + pad, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(arena, sh.byte_lo, PAYLOAD_SEED)
    off = torch.from_numpy(sh.local_off.astype(np.int64)).to(dev)
    ln = torch.from_numpy(sh.lens.view(np.int32)).to(dev)
    return arena, off, ln, sh, desc


def global_lengths(name):
    """The c2 / c4 length lists (rank-independent, for strong scaling)."""
    import numpy as np
    if name == "c2":
        return wal_unit_lengths(1048576)
    rng = np.random.default_rng(0xC0FFEE)
    kk = np.arange(1, 2049, dtype=np.float64)
    cdf = np.cumsum(kk ** -1.1)
    cdf /= cdf[-1]
    k = np.minimum(np.searchsorted(cdf, rng.random(1048576), side="right") + 1, 2048)
    return (32 * k).astype(np.uint32)


def main():
    global SETTLE
    args = parse()
    SETTLE = args.settle
    single = [m for m in ("wal", "c1", "e2e", "sweep", "table", "hash", "long", "wal_device") if getattr(args, m)]
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if single and args.gpus > 1:
        raise SystemExit(f"--{single[0].replace('_', '-')} is a single-GPU diagnostic; run it with --gpus 1")
    from lvgpu import shard
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` without torchrun: start the N ranks here
        # (one process per GPU, env:// rendezvous on 127.0.0.1).  This process
        # never touches a GPU; rank 0's JSON line is the output.
        sys.exit(shard.self_launch(__file__, sys.argv[1:], args.gpus))
    if args.wal:
        return wal_bench(args)
    if args.c1:
        return c1_sweep(args)
    if args.e2e:
        return e2e(args)
    if args.sweep:
        return sweep_bench(args)
    if args.table:
        return table_bench(args)
    if args.hash:
        return hash_bench(args)
    if args.long:
        return long_bench(args)
    if args.wal_device:
        return wal_device_bench(args)
    world, rank, local = shard.world_from_env(args.gpus)
    # --as-rank/--as-world: a single process rebuilds rank R's shard of a
    # W-rank job (the PMC child pass of measure_traffic runs this way).
    shard_rank, shard_world = (args.as_rank, args.as_world) if args.as_world > 1 else (rank, world)
    if args.as_world > 1 and world > 1:
        raise SystemExit("--as-rank/--as-world replay one rank's shard in a single process")
    import torch
    import lvgpu

    dist = None
    # LVGPU_BENCH_BACKEND=gloo rehearses the N>1 path on a box with fewer GPUs
    # than ranks (ranks share devices round-robin; RCCL refuses two ranks on
    # one device).  The data path has no collective either way.
    backend = os.environ.get("LVGPU_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    elif world > 1 and local >= torch.cuda.device_count():
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but only {torch.cuda.device_count()} visible GPUs "
                         f"(--gpus {args.gpus} needs one GPU per rank; LVGPU_BENCH_BACKEND=gloo to share)")
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        with _stdout_to_stderr():  # the backends' C++ chatter must not reach the one JSON line's stdout
            if backend == "nccl":
                dist.init_process_group(backend, device_id=torch.device(f"cuda:{local}"))
            else:
                dist.init_process_group(backend)
                dist.barrier()  # gloo prints its peer connections lazily
        if dist.get_world_size() != world:
            raise SystemExit(f"process group has {dist.get_world_size()} ranks, expected {world}")
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    lvgpu.device_init()

    if args.scaling == "strong":
        arena, off, ln, sh, desc = build_shard(torch, lvgpu, args, dev, shard_rank, shard_world)
        nbytes, n = sh.payload_bytes, sh.n
    else:
        arena, off, ln, nbytes, desc = build_workload(torch, lvgpu, args.workload, dev, shard_rank, args.blocks)
        n = off.numel()
    out = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()
    strided = args.api == "strided" and args.workload in ("c3", "c5")

    if n == 0:
        def step():
            pass
    elif strided:
        def step():
            lvgpu.batch_strided(arena, 4096, 4096, n, out=out, stream=stream, group=args.group)
    else:
        def step():
            lvgpu.batch(arena, off, ln, out=out, stream=stream, group=args.group)

    settle_info = settle(torch, step, stream) if args.settle and n else None
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # Timed region (value): K steps between barrier + synchronize, nothing
    # else on the stream, max over ranks (lvgpu.shard.timed_steps, the code
    # the gloo test drives).  A timestamp event between launches costs ~3 %
    # of the step time on MI355X, so the per-launch HIP events for
    # roofline.achieved are taken in a second pass of the same K steps, right
    # after, on the launch stream.
    el_own, el = shard.timed_steps(
        step, args.steps, torch.cuda.synchronize, dist,
        lambda x: torch.tensor([x], dtype=torch.float64, device=dev if backend == "nccl" else "cpu"))
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    torch.cuda.synchronize()
    for s, e in evs:
        s.record(stream)
        step()
        e.record(stream)
    torch.cuda.synchronize()
    kern_seq = [s.elapsed_time(e) for s, e in evs]
    kern_ms = sorted(kern_seq)
    if os.environ.get("LVGPU_BENCH_TRACE"):
        print("per-launch ms:", " ".join(f"{x:.4f}" for x in kern_seq), file=sys.stderr)
    kern_avg_ms = sum(kern_ms) / len(kern_ms)
    # per-GPU figures: each rank's own timed-pass rate and kernel rate
    props = torch.cuda.get_device_properties(dev)
    own = {"rank": rank, "device": local,
           "pci_bus_id": f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}",
           "gpu_uuid": str(getattr(props, "uuid", "")), "hostname": socket.gethostname(),
           "payload_bytes": nbytes,
           "GiB_per_s": round(nbytes * args.steps / 2**30 / el_own, 2),
           "kernel_GB_per_s": round(nbytes / (kern_avg_ms * 1e-3) / 1e9, 1),
           "frac_of_8TBps": round(nbytes / (kern_avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    per_rank = shard.gather_ranks(own, dist, world)
    agg = shard.aggregate(per_rank, args.steps, el)
    value = agg["GiB_per_s"]
    achieved_gbs = nbytes / (kern_avg_ms * 1e-3) / 1e9
    kernel = lvgpu.last_kernel()

    result = None
    if rank == 0:
        cpu = None
        # after the timed region: on rank 0 at every N (the other ranks wait
        # at the closing barrier), over rank 0's own shard
        if args.cpu_seconds > 0:
            cpu, crcs, k = cpu_baseline(torch, arena, off, ln, args.cpu_seconds)
            got = out[:k].cpu().numpy().view("uint32")
            if not (got == crcs).all():
                raise SystemExit("bench parity check failed: GPU CRCs differ from the oracle on the sample")
        traffic, tsrc = (None, "not collected")
        if args.traffic == "auto":
            traffic, tsrc = measure_traffic(args, shard_rank, shard_world)
        result = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world,
            "world_size": dist.get_world_size() if dist else 1,
            "launcher": os.environ.get("LVGPU_LAUNCHER", "torch.distributed.run" if world > 1 else "single process"),
            "backend": backend if world > 1 else None,
            "distinct_devices": len({(r["hostname"], r["pci_bus_id"]) for r in per_rank}),
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (splitmix64 payload generated in HBM)",
            "config": {"workload": desc, "buffers_per_gpu": n, "bytes_per_gpu": nbytes,
                       "total_bytes_per_step": agg["total_bytes_per_step"],
                       "api": "lv_crc32c_batch_strided" if strided else "lv_crc32c_batch_device",
                       "parallelism": (f"dp{world} (independent shards, no collective)" if args.scaling == "weak"
                                       else f"dp{world} (one global batch split into contiguous rank ranges, "
                                            f"no collective)")},
            "hbm_peak_frac": round(value * 2**30 / world / 1e9 / HBM_PEAK_GBS, 4),
            "settle": settle_info,
            "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                         "traffic": None if traffic is None else round(traffic), "traffic_source": tsrc,
                         "kernel": "lvk::" + kernel if strided else
                                   "lv_crc32c_batch_device step: lvk::sort_{hist,scan,scatter} + "
                                   "lvk::crc32c_classes_kernel",
                         "kernel_ms_avg": round(kern_avg_ms, 4),
                         "kernel_ms_min": round(kern_ms[0], 4),
                         "kernel_ms_p50": round(kern_ms[len(kern_ms) // 2], 4),
                         "kernel_ms_max": round(kern_ms[-1], 4), "bytes_per_launch": nbytes,
                         "timing": "HIP events around each of K launches on the launch stream, in a second "
                                   "pass of the K timed steps"},
            "cpu_baseline": cpu,
            "per_gpu": per_rank,
            "load_imbalance": round(agg["imbalance"], 4),
        }
        print(json.dumps(result), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
