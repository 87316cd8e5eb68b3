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
    p.add_argument("--host-placement", default="gpu-local", choices=["gpu-local", "float"],
                   help="--wal: confine the process to the CPUs local to the GPU (its PCI function's "
                        "local_cpulist, as numactl --cpunodebind would) before the log is allocated, or leave it "
                        "where the OS puts it")
    p.add_argument("--variants", action="store_true",
                   help="SURVEY 8d's config variants through the offsets API: C2 with the writer's seeds "
                        "type_crc[t] over payload only (masked), C2 heavy (uniform 0-32761 B payloads, 16 GiB), "
                        "C4 misaligned (L - r, r in [0, 31]); one JSON line")
    p.add_argument("--wal-device", action="store_true",
                   help="SURVEY 8f row 1 in HBM: lv_wal_scan_device (framing + CRC) of a ~1 GiB log already on "
                        "the GPU; one JSON line with a roofline")
    p.add_argument("--as-rank", type=int, default=0, help=argparse.SUPPRESS)
    p.add_argument("--as-world", type=int, default=1, help=argparse.SUPPRESS)
    p.add_argument("--c5-strong", default="auto", choices=["auto", "off"],
                   help="auto: the default C3 line also times BASELINE configs[4] (64 GiB of 4 KiB blocks split "
                        "across the ranks) as its `c5_strong` sub-record")
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
    return wal_units_typed(n)[0] + 1


def wal_units_typed(n):
    """(fragment length, record type) of the first n physical records the
    reference writer emits for Random(301).skewed(17) records
    (log_writer.rs:62-110: FULL 1, FIRST 2, MIDDLE 3, LAST 4; trailers of
    < 7 B skipped), i.e. the writer's CRC calls extend(type_crc[t], fragment)
    (log_writer.rs:123).  The Park-Miller generator is random.rs:19-70."""
    import numpy as np
    B, H = 32768, 7
    frags = np.empty(n, dtype=np.uint32)
    types = np.empty(n, dtype=np.uint32)
    m, state, block_off = 0, 301 & 0x7FFFFFFF, 0

    def nxt():
        nonlocal state
        prod = state * 16807
        v = ((prod >> 31) + (prod & 2147483647)) & 0xFFFFFFFF
        if v > 2147483647:
            v -= 2147483647
        state = v
        return v
    while m < n:
        r = 1 << (nxt() % 18)
        left, begin = nxt() % r, True
        while m < n:
            if B - block_off < H:
                block_off = 0
            frag = min(left, B - block_off - H)
            end = frag == left
            frags[m] = frag
            types[m] = 1 if begin and end else 2 if begin else 4 if end else 3
            m += 1
            block_off += H + frag
            left -= frag
            begin = False
            if end:
                break
    return frags, types


def variants_bench(args):
    """SURVEY 8d's config variants, each through lv_crc32c_batch_device (sort
    + class kernel) in HBM: (a) C2 as the WAL writer calls it --
    mask(extend(type_crc[t], fragment)) over the payload alone, seeds in a
    device array, LV_CRC_MASK (log_writer.rs:112-125); (b) C2 heavy: 1,048,576
    units of 1 + U[0, 32761] bytes (16 GiB); (c) C4 misaligned: the C4 lengths
    L - r, r uniform in [0, 31], byte-packed.  HIP-event mean per call after
    settle + warmup; the first and last 1,000 buffers of each checked against
    the oracle (seeds and mask included)."""
    import numpy as np
    import torch
    import lvgpu
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import wal_oracle as W
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    lvgpu.device_init()
    L = W.lib()
    type_crc = np.array([lvgpu.value(bytes([t])) for t in range(5)], dtype=np.uint32)  # log_writer.rs:136-142
    rng = np.random.default_rng(0x5EED)
    cases = []
    u, t = wal_units_typed(1048576)
    cases.append(("c2_writer_seeded_masked", u, type_crc[t], True,
                  "C2 fragments (payload only) with seed type_crc[t] and LV_CRC_MASK: the writer's call"))
    cases.append(("c2_heavy", (1 + rng.integers(0, 32762, 1048576)).astype(np.uint32), None, False,
                  "1,048,576 units of 1 + U[0, 32761] B (mean 16,382 B), byte-packed"))
    kk = np.arange(1, 2049, dtype=np.float64)
    cdf = np.cumsum(kk ** -1.1)
    cdf /= cdf[-1]
    k = np.minimum(np.searchsorted(cdf, np.random.default_rng(0xC0FFEE).random(1048576), side="right") + 1, 2048)
    c4 = (32 * k - rng.integers(0, 32, k.size)).astype(np.uint32)
    cases.append(("c4_misaligned", c4, None, False, "C4 lengths L - r, r ~ U[0, 31], byte-packed"))
    steps, warm = max(20, min(args.steps, 100)), max(10, min(args.warmup, 50))
    rows = []
    for name, lens, seeds, masked, desc in cases:
        n = lens.size
        offs = np.zeros(n, dtype=np.uint64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        total = int(offs[-1] + lens[-1])
        arena = torch.empty(total + 64, dtype=torch.uint8, device=dev)
        lvgpu.fill_splitmix(arena, 0, PAYLOAD_SEED)
        o = torch.from_numpy(offs.astype(np.int64)).to(dev)
        ln = torch.from_numpy(lens.view(np.int32)).to(dev)
        sd = None if seeds is None else torch.from_numpy(seeds.view(np.int32)).to(dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        ws = torch.empty(lvgpu.workspace_bytes(n), dtype=torch.uint8, device=dev)
        fn = lambda: lvgpu.batch_ws(arena, o, ln, ws, seed=sd, out=out, masked=masked)  # noqa: E731
        p50, avg = _event_times(torch, fn, steps, warm)
        out.fill_(0)
        fn()
        kern = lvgpu.last_kernel()
        got = out.cpu().numpy().view(np.uint32)
        for lo, hi in ((0, 1000), (n - 1000, n)):
            a0, a1 = int(offs[lo]), int(offs[hi - 1] + lens[hi - 1])
            host = arena[a0:a1].cpu().numpy()
            ho = (offs[lo:hi] - a0).astype(np.uint64)
            hl = np.ascontiguousarray(lens[lo:hi])
            hs = None if seeds is None else np.ascontiguousarray(seeds[lo:hi])
            want = np.zeros(hi - lo, dtype=np.uint32)
            L.oracle_batch(host.ctypes.data, ho.ctypes.data, hl.ctypes.data,
                           None if hs is None else hs.ctypes.data, want.ctypes.data, hi - lo, 1 if masked else 0)
            if not np.array_equal(got[lo:hi], want):
                raise SystemExit(f"variants parity check failed ({name}, buffers {lo}..{hi})")
        gbs = total / (avg * 1e-3) / 1e9
        rows.append({"variant": name, "config": desc, "buffers": n, "payload_bytes": total,
                     "GB_per_s": round(gbs, 1), "GiB_per_s": round(total / (avg * 1e-3) / 2**30, 2),
                     "frac_of_8TBps": round(gbs / HBM_PEAK_GBS, 4), "ms_avg": round(avg, 4),
                     "ms_p50": round(p50, 4), "kernels": kern,
                     "parity": "first and last 1,000 buffers == oracle_batch (seeds, mask)"})
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
        del arena, o, ln, sd, out, ws
        torch.cuda.empty_cache()
    res = {"metric": "SURVEY 8d config variants, device-resident batched CRC32C (offsets API)", "unit": "GB/s",
           "results": rows, "timing": "HIP events around each call (every kernel of the call), mean after "
           "settle + warmup", "data": "synthetic splitmix64 payload in HBM"}
    print(json.dumps(res), flush=True)
    return res


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
           "--traffic", "off", "--no-settle", "--c5-strong", "off", "--workload", args.workload, "--api", args.api,
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


def pmc_per_kernel(bench_args, counter, keep=None, last=None):
    """Child process: one rocprofv3 --pmc pass of `counter` (FETCH_SIZE or
    WRITE_SIZE, kernel counters only, its own run) over bench.py with
    `bench_args`; returns {kernel: mean bytes per launch} for the lvk::
    kernels (FETCH_SIZE doubled per the gfx950 correction, WRITE_SIZE as read:
    MI355X_MICROARCH.md §HBM), or (None, reason)."""
    import glob
    import shutil
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3")
    if exe is None:
        return None, "rocprofv3 not found"
    if any(k.startswith("ROCPROF") for k in os.environ):
        return None, "skipped (running under rocprofv3)"
    out = tempfile.mkdtemp(prefix="lvgpu_pmc_", dir="/tmp")
    cmd = [exe, "--pmc", counter, "--output-format", "csv", "-d", out, "-o", "pmc", "--",
           sys.executable, os.path.abspath(__file__)] + bench_args
    env = dict(os.environ, TMPDIR="/tmp")
    try:
        subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                       timeout=300, check=True)
    except Exception as e:  # noqa: BLE001 - report, never fail the bench on the profiler
        shutil.rmtree(out, ignore_errors=True)
        return None, f"rocprofv3 pass failed: {e}"
    per = {}
    for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
        per.update(read_pmc_per_kernel(f, counter, keep, last))
    shutil.rmtree(out, ignore_errors=True)
    if not per:
        return None, "no lvk:: kernel in the pass"
    return per, f"rocprofv3 --pmc {counter}, mean per launch"


def read_pmc_per_kernel(path, counter, keep=None, last=None):
    """{kernel: mean bytes per launch} of `counter` over the lvk:: kernels of a
    rocprofv3 counter CSV (fill kernels excluded; FETCH_SIZE KiB doubled for
    gfx950's half-counted wide reads, WRITE_SIZE KiB as read).  `keep`: only
    these kernel names; `last`: only each name's last `last` launches (by
    dispatch id), so set-up calls before the timed ones do not count."""
    import collections
    import csv
    scale = 2.0 * 1024.0 if counter == "FETCH_SIZE" else 1024.0
    per = collections.defaultdict(list)
    with open(path) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "")
            if "lvk::" in name and "fill_" not in name and row.get("Counter_Name") == counter:
                k = name.split("(")[0].replace("void ", "")
                if keep is None or k in keep:
                    per[k].append((int(row.get("Dispatch_Id") or 0), float(row["Counter_Value"]) * scale))
    out = {}
    for k, v in per.items():
        v = [x for _, x in sorted(v)][-last:] if last else [x for _, x in v]
        out[k] = sum(v) / len(v)
    return out


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


def cpu_loop_baseline(pass_fn, n, seconds, sample, unit_scale=2**30, unit="GiB/s", threads=16):
    """A CPU baseline for the SURVEY 8f lines: `pass_fn(lo, hi)` runs the
    oracle's restatement of the reference loop over items [lo, hi) of the
    same workload once and returns the bytes (or keys) it covered.  One
    thread for `seconds` (the reference callers are single-threaded), then
    the box's 16-thread CPU share over equal slices for seconds / 4, for
    context (ctypes drops the GIL inside the C calls)."""
    import threading

    def run(lo, hi, secs, out):
        done, t0 = 0, time.perf_counter()
        while True:
            done += pass_fn(lo, hi)
            el = time.perf_counter() - t0
            if el >= secs:
                break
        out.append((done, el))
    single = []
    run(0, n, seconds, single)
    bounds = [n * t // threads for t in range(threads + 1)]
    agg, th = [], []
    for t in range(threads):
        if bounds[t + 1] > bounds[t]:
            th.append(threading.Thread(target=run, args=(bounds[t], bounds[t + 1], max(1.0, seconds / 4), agg)))
    for t in th:
        t.start()
    for t in th:
        t.join()
    d1, e1 = single[0]
    return {"value": round(d1 / unit_scale / e1, 3), "unit": unit, "cores": 1, "kind": "port",
            "sample": f"{sample}; {e1:.1f} s on 1 thread",
            "all_cores": {"value": round(sum(d / e for d, e in agg) / unit_scale, 2), "unit": unit,
                          "threads": len(th), "note": "same work split over the box's 16-thread CPU share"},
            "host_cpu": _cpu_model(), "host_nproc": os.cpu_count()}


def wal_oracle_check(log, expect_records):
    """The oracle's whole-log verify (oracle_wal_verify, log_reader.rs:271-364)
    finds every record intact: the stored header CRCs equal the oracle's."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import wal_oracle as W
    mm = ctypes.c_uint64()
    ok = W.lib().oracle_wal_verify(log.ctypes.data, int(log.size), ctypes.byref(mm), None)
    if ok != expect_records or mm.value:
        raise SystemExit(f"WAL oracle verify found {ok} good / {mm.value} bad records, expected {expect_records}")


def wal_cpu_baseline(log, seconds, expect_records):
    """The reference reader's verify (log_reader.rs:271-364: 32 KiB reads,
    header framing, unmask(header) == value([type || payload]) per record)
    restated in C (oracle_wal_verify) over the same log, in GB/s of log.
    Blocks are independent, so the 16-thread figure splits at block bounds."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import wal_oracle as W
    L = W.lib()
    size = int(log.size)
    base = log.ctypes.data
    nblk = (size + 32767) // 32768
    mm = ctypes.c_uint64()
    ok = L.oracle_wal_verify(base, size, ctypes.byref(mm), None)
    if ok != expect_records or mm.value:
        raise SystemExit(f"WAL cpu baseline: oracle verify found {ok} good / {mm.value} bad records, "
                         f"expected {expect_records}")

    def one(lo, hi):
        b0, b1 = lo * 32768, min(size, hi * 32768)
        L.oracle_wal_verify(base + b0, b1 - b0, None, None)
        return b1 - b0
    return cpu_loop_baseline(one, nblk, seconds, f"the whole {size / 2**30:.2f} GiB log, oracle_wal_verify "
                             f"(framing + CRC of log_reader.rs:271-364)", unit_scale=1e9, unit="GB/s")


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
    sort + class kernel; with a uniform hint the class kernel alone), and (c)
    the aligned layout through the offsets API with LV_HINT_ALIGNED16 (the
    uniform-block kernel reading each start from the offsets).  HIP-event mean over the timed launches; 64 blocks
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
        hint = lvgpu.BatchHint(n * bl, bl, 1)  # uniform, nothing splits: the class kernel alone, no sort
        # the strided layout through the offsets API with LV_HINT_ALIGNED16: the blocks kernel, gathering
        o_al = torch.arange(n, dtype=torch.int64, device=dev) * bl
        hint_al = lvgpu.BatchHint(n * bl, bl, lvgpu.HINT_UNIFORM | lvgpu.HINT_ALIGNED16)
        for api, fn in (("strided", lambda: lvgpu.batch_strided(arena, bl, bl, n, out=out)),
                        ("offsets", lambda: lvgpu.batch_ws(arena, o, ln, ws, out=out)),
                        ("offsets_hint", lambda: lvgpu.batch_hint(arena, o, ln, hint, out=out, workspace=ws)),
                        ("offsets_hint_aligned",
                         lambda: lvgpu.batch_hint(arena, o_al, ln, hint_al, out=out, workspace=ws))):
            out.fill_(0)
            _, avg = _event_times(torch, fn, steps, warm)
            fn()
            kern = lvgpu.last_kernel()
            lvgpu.batch_check()  # the hints were exact: no violation recorded on the device
            k = 64
            base = 0 if api in ("strided", "offsets_hint_aligned") else 13
            row.setdefault("kernels", {})[api] = kern
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
        del out, o, o_al, ln, ws
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
        hint = lvgpu.BatchHint(n * bl, bl, 1)  # uniform: what a caller that knows its lengths passes
        # ... and that knows its buffers start 16-B aligned (the strided API's kernels, gathering)
        hint_al = lvgpu.BatchHint(n * bl, bl, lvgpu.HINT_UNIFORM | lvgpu.HINT_ALIGNED16)
        for api, fn in (("strided", lambda: lvgpu.batch_strided(arena, bl, bl, n, out=out)),
                        ("offsets", lambda: lvgpu.batch_ws(arena, o, ln, ws, out=out)),
                        ("offsets_hint", lambda: lvgpu.batch_hint(arena, o, ln, hint, out=out, workspace=ws)),
                        ("offsets_hint_aligned",
                         lambda: lvgpu.batch_hint(arena, o, ln, hint_al, out=out, workspace=ws))):
            p50, avg = _event_times(torch, fn, max(20, min(args.steps, 100)), max(10, min(args.warmup, 50)))
            fn()
            kern = lvgpu.last_kernel()
            lvgpu.batch_check()  # the hints were exact: no violation recorded on the device
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
        # every record: the GPU value([type||payload]) == unmask(its header's
        # stored CRC); the oracle's whole-log verify (wal_oracle_check below)
        # pins the stored CRCs to the oracle's, so the two give every record
        hc = h_hdr.astype(np.int64)
        stored = (log[hc].astype(np.uint32) | (log[hc + 1].astype(np.uint32) << 8)
                  | (log[hc + 2].astype(np.uint32) << 16) | (log[hc + 3].astype(np.uint32) << 24))
        r = (stored - np.uint32(0xa282ead8)).astype(np.uint32)
        unm = ((r >> np.uint32(17)) | (r << np.uint32(15))).astype(np.uint32)  # crc32c.rs:59-63
        okst = ((h_info >> 8) & 0xff) == 0
        if not np.array_equal(h_crc[okst], unm[okst]) or not okst.all():
            raise SystemExit("WAL device scan: a record's CRC differs from its header")
        parity = ("every record's GPU CRC == unmask(its header CRC), and the oracle's whole-log verify "
                  "(oracle_wal_verify) accepts every header; first 2000 records also vs oracle value()")
    variant = os.environ.get("LVGPU_EXPERIMENT") == "1"
    if not variant:  # the oracle's verify of the whole log, untimed (the cpu_baseline below times it)
        wal_oracle_check(log, cap)
    # HBM traffic per call: FETCH_SIZE and WRITE_SIZE per kernel,
    # each in its own child pass over the same log and scan
    traffic = None
    if args.traffic == "auto":
        child = ["--wal-device", "--steps", "10", "--warmup", "5", "--cpu-seconds", "0", "--traffic", "off",
                 "--no-settle"] + (["--blocks", str(args.blocks)] if args.blocks else [])
        # the scan's five kernels, the timed launches only (the log's encode
        # ran the seeded batch path on the same device first)
        keep = {"lvk::wal_hist", "lvk::sort_scan", "lvk::wal_scatter", "lvk::crc32c_classes_kernel<false>",
                "lvk::wal_unsort"}
        fetch, fsrc = pmc_per_kernel(child, "FETCH_SIZE", keep, 10)
        write, wsrc = pmc_per_kernel(child, "WRITE_SIZE", keep, 10)
        if isinstance(fetch, dict):
            traffic = {"fetch_bytes_per_call": round(sum(fetch.values())),
                       "fetch_over_log_bytes": round(sum(fetch.values()) / log.size, 4),
                       "per_kernel_fetch": {k: round(v) for k, v in fetch.items()},
                       "source": fsrc + " (x2 gfx950 correction); the call's kernels summed"}
            if isinstance(write, dict):
                traffic["write_bytes_per_call"] = round(sum(write.values()))
                traffic["per_kernel_write"] = {k: round(v) for k, v in write.items()}
        else:
            traffic = {"error": fsrc}
    cpu = wal_cpu_baseline(log, args.cpu_seconds, cap) if args.cpu_seconds > 0 and not variant else None
    gbs = log.size / (avg * 1e-3) / 1e9
    res = {"metric": "device-resident WAL verify scan (framing + CRC of every record), HBM", "unit": "GB/s",
           "log_bytes": int(log.size), "records": int(sizes.size), "physical_records": cap,
           "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(gbs / HBM_PEAK_GBS, 4), "ms_avg": round(avg, 4), "ms_p50": round(p50, 4),
                        "bytes_per_call": int(log.size),
                        "kernels": lvgpu.last_kernel(),
                        "traffic": None if not traffic else traffic.get("fetch_bytes_per_call"),
                        "traffic_detail": traffic},
           "api": "lv_wal_scan_device", "parity": parity, "cpu_baseline": cpu,
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
    host_e2e = table_host_e2e(torch, T, f, offs, sizes) if not variant else None
    cpu = table_cpu_baseline(f, offs, sizes, unit, args.cpu_seconds) if args.cpu_seconds > 0 and not variant else None
    res = {"metric": "SSTable block trailer seal / verify, device-resident", "unit": "GiB/s",
           "blocks": n, "bytes_per_call": unit, "table_bytes": total,
           "seal": {"GiB_per_s": round(unit / 2**30 / (seal_avg * 1e-3), 1), "ms_avg": round(seal_avg, 4),
                    "ms_p50": round(seal_p50, 4), "frac_of_8TBps": round(unit / (seal_avg * 1e-3) / 8e12, 4)},
           "verify": {"GiB_per_s": round(unit / 2**30 / (ver_avg * 1e-3), 1), "ms_avg": round(ver_avg, 4),
                      "ms_p50": round(ver_p50, 4), "frac_of_8TBps": round(unit / (ver_avg * 1e-3) / 8e12, 4)},
           "timing": "HIP events around each call (CRC batch + trailer kernels)", "parity": ("first 2000 blocks' CRCs vs oracle value(); every sealed trailer vs the oracle's "
                      "verify (oracle_units_verify, in the cpu_baseline pass)" if cpu else "first 2000 blocks vs oracle"),
           "host_e2e": host_e2e, "cpu_baseline": cpu,
           "data": "synthetic splitmix64 contents in HBM"}
    print(json.dumps(res), flush=True)
    return res


def table_host_e2e(torch, T, f, offs, sizes, reps=5):
    """lv_sst_verify_blocks_host end to end on the same sealed table in host
    memory (H2D of the file + handles through the device's cached host path,
    one verify launch, D2H of the statuses): pageable and pinned input, median
    of `reps` calls, in GiB/s of table bytes."""
    import numpy as np
    L = T._bind()
    n = int(offs.size)
    hh = np.ascontiguousarray(np.stack([offs, sizes], axis=1).astype(np.uint64))
    st = np.zeros(n, dtype=np.uint32)
    page = f.cpu().numpy()
    pin = torch.empty(page.size, dtype=torch.uint8, pin_memory=True)
    pin.numpy()[:] = page
    res = {}
    for name, arr in (("pageable", page), ("pinned", pin.numpy())):
        ts = []
        for r in range(reps + 1):
            st[:] = 99
            t0 = time.perf_counter()
            rc = L.lv_sst_verify_blocks_host(arr.ctypes.data, arr.size, hh.ctypes.data, n, st.ctypes.data, 0)
            el = time.perf_counter() - t0
            if rc or not (st == T.BLOCK_OK).all():
                raise SystemExit(f"lv_sst_verify_blocks_host failed ({name}): rc {rc}")
            if r:
                ts.append(el)
        med = sorted(ts)[len(ts) // 2]
        res[name] = {"GiB_per_s": round(page.size / 2**30 / med, 2), "ms": round(med * 1e3, 2)}
    res["api"] = "lv_sst_verify_blocks_host (H2D + verify + D2H of statuses)"
    return res


def table_cpu_baseline(f, offs, sizes, unit_bytes, seconds):
    """Per-block trailer verify and seal on one host core over the same
    (sealed) table copied to host memory: value(contents || type) against
    unmask(LE32 after it) / mask(extend(value(contents), [type])) written
    after the type (oracle_units_verify / oracle_units_seal), in GiB/s of
    contents + type, like the GPU line."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import wal_oracle as W
    L = W.lib()
    host = f.cpu().numpy().copy()
    uo = offs.astype(np.uint64)
    ul = (sizes + 1).astype(np.uint32)
    co = (offs + sizes + 1).astype(np.uint64)
    sz = sizes.astype(np.uint32)
    n = int(offs.size)
    if L.oracle_units_verify(host.ctypes.data, uo.ctypes.data, ul.ctypes.data, co.ctypes.data, n):
        raise SystemExit("table cpu baseline: the oracle rejects a trailer the GPU sealed")
    per_block = ul.astype(np.uint64)
    csum = np.concatenate([[0], np.cumsum(per_block)])

    def verify(lo, hi):
        L.oracle_units_verify(host.ctypes.data, uo[lo:].ctypes.data, ul[lo:].ctypes.data, co[lo:].ctypes.data, hi - lo)
        return int(csum[hi] - csum[lo])

    def seal(lo, hi):
        L.oracle_units_seal(host.ctypes.data, uo[lo:].ctypes.data, sz[lo:].ctypes.data, hi - lo)
        return int(csum[hi] - csum[lo])
    samp = f"the whole table ({unit_bytes / 2**30:.2f} GiB of contents + type, {n} blocks) in host memory"
    v = cpu_loop_baseline(verify, n, seconds, samp + ", oracle_units_verify: unmask(trailer) == value(contents||type)")
    s = cpu_loop_baseline(seal, n, seconds / 2, samp + ", oracle_units_seal: mask(extend(value(contents), type))")
    if L.oracle_units_verify(host.ctypes.data, uo.ctypes.data, ul.ctypes.data, co.ctypes.data, n):
        raise SystemExit("table cpu baseline: the oracle seal differs from the GPU seal")
    return {"verify": v, "seal": s}


# VALU issue of the hash kernels.  MI355X: 256 CUs x 4
# SIMDs at up to 2.4 GHz (MI355X_MICROARCH.md).  Measured on this part
# (tools/pmc_calib.hip, profiles/r05/valu/): SQ_INSTS_VALU is the exact
# whole-GPU count of wave-level VALU instructions, and a dependent stream of
# simple 32-bit wave64 ops issues one per 2.44 SIMD cycles at the 2.4 GHz
# clock (v_mul_lo_u32: 4.56) -- so the VALU peak is 1,024 x 2.4e9 / 2.44
# wave instructions per second, every instruction priced as a simple op.
VALU_SIMDS, VALU_CLOCK_HZ, VALU_CYCLES = 1024, 2.4e9, 2.44
SQ_VALU_SCALE = 1.0


def hash_api_of(kernel_name):
    """The hash API a hash_kernel<Meta> dispatch serves, by its template
    argument (every variant's parameter list holds "unsigned int")."""
    if "PackedMeta<unsigned int>" in kernel_name:
        return "packed_u32"
    if "PackedMeta<unsigned long>" in kernel_name:
        return "packed_u64"
    return "offsets"


def measure_hash_valu(args):
    """Child process: rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES over a short hash
    run (kernel counters only).  Returns {kernel api: VALU instructions per
    launch} or (None, reason)."""
    import collections
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3")
    if exe is None:
        return None, "rocprofv3 not found"
    if any(k.startswith("ROCPROF") for k in os.environ):
        return None, "skipped (running under rocprofv3)"
    out = tempfile.mkdtemp(prefix="lvgpu_valu_", dir="/tmp")
    cmd = [exe, "--pmc", "SQ_INSTS_VALU", "SQ_WAVES", "--output-format", "csv", "-d", out, "-o", "pmc", "--",
           sys.executable, os.path.abspath(__file__), "--hash", "--steps", "3", "--warmup", "1", "--cpu-seconds", "0",
           "--traffic", "off"]
    if args.blocks:
        cmd += ["--blocks", str(args.blocks)]
    env = dict(os.environ, TMPDIR="/tmp")
    try:
        subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                       timeout=300, check=True)
    except Exception as e:  # noqa: BLE001 - report, never fail the bench on the profiler
        return None, f"rocprofv3 pass failed: {e}"
    per = collections.defaultdict(list)
    for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if "hash_kernel" in name and row.get("Counter_Name") == "SQ_INSTS_VALU":
                    api = hash_api_of(name)
                    per[api].append(float(row["Counter_Value"]))
    shutil.rmtree(out, ignore_errors=True)
    if not per:
        return None, "no hash_kernel counters in the pass"
    return {k: SQ_VALU_SCALE * sum(v) / len(v) for k, v in per.items()}, \
        "rocprofv3 --pmc SQ_INSTS_VALU (its own pass), mean per launch"


def hash_rooflines(key_bytes, ms, valu_instr, moved_bytes):
    """The hash line's two bounds: HBM -- `frac` by key bytes,
    `frac_all_bytes` by every byte the API moves (keys, metadata, output) --
    and VALU issue (instructions x 2.44 cycles over 1,024 SIMDs at 2.4 GHz).
    `roofline` is the one closer to its peak, comparing like with like: the
    HBM `frac` it reports (key bytes, SURVEY 8d's algorithmic bytes) against
    the VALU `frac` (the rule and the reported number agree)."""
    g = key_bytes / (ms * 1e-3) / 1e9
    ga = moved_bytes / (ms * 1e-3) / 1e9
    hbm = {"bound": "hbm", "achieved": round(g, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(g / HBM_PEAK_GBS, 4), "bytes_per_launch": key_bytes,
           "algorithmic_bytes": "key bytes only (SURVEY 8d)",
           "frac_all_bytes": round(ga / HBM_PEAK_GBS, 4), "all_bytes_per_launch": moved_bytes,
           "selection": "roofline = the bound with the larger frac: HBM frac by key bytes vs VALU frac"}
    if valu_instr is None:
        return hbm, hbm, None
    peak_ips = VALU_SIMDS * VALU_CLOCK_HZ / VALU_CYCLES  # wave-level VALU instructions per second
    ips = valu_instr / (ms * 1e-3)
    valu = {"bound": "valu", "achieved": round(ips / 1e12, 4), "peak": round(peak_ips / 1e12, 4),
            "unit": "T wave-VALU instr/s", "frac": round(ips / peak_ips, 4),
            "instr_per_launch": round(valu_instr), "cycles_per_instr": VALU_CYCLES}
    return (valu if valu["frac"] > hbm["frac"] else hbm), hbm, valu


def hash_cpu_baseline(arena, offs, lens, seconds):
    """hash.rs:20-51 per key on one host core (oracle_hash_batch) over the
    same byte-packed keys copied to host memory, in G keys/s."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import wal_oracle as W
    L = W.lib()
    host = arena.cpu().numpy()
    n = int(offs.size)
    outb = np.zeros(n, dtype=np.uint32)
    keyb = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)])

    def one(lo, hi):
        L.oracle_hash_batch(host.ctypes.data, offs[lo:].ctypes.data, lens[lo:].ctypes.data, None,
                            outb[lo:].ctypes.data, hi - lo)
        return hi - lo
    r = cpu_loop_baseline(one, n, seconds, f"all {n} keys ({int(keyb[-1]) / 1e9:.3f} GB) in host memory, "
                          f"oracle_hash_batch (hash.rs:20-51, seed 0 as cache.rs:182/:395)", unit_scale=1e9, unit="Gkeys/s")
    r["key_GB_per_s"] = round(r["value"] * float(keyb[-1]) / n, 3)
    return r


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
    variant = lvgpu.experiment_variant()  # timing studies of experiment variants (wrong hashes by design) skip parity
    if not variant and not np.array_equal(out[:k].cpu().numpy().view(np.uint32), want):
        raise SystemExit("hash bench parity check failed")
    # packed keys (lv_hash_batch_packed): the same keys described by n + 1
    # bounds of 8 or 4 bytes instead of 12 B of offset + length per key
    packed = {}
    bnd = np.concatenate([offs, [total]]).astype(np.int64)
    for width, dt in ((8, torch.int64), (4, torch.int32)):
        b = torch.from_numpy(bnd.astype(np.int64 if width == 8 else np.int32)).to(dev)
        pp50, pavg = _event_times(torch, lambda: H.hash_batch_packed(arena, b, out=out, shard=True),
                                  args.steps, args.warmup)
        H.hash_batch_packed(arena, b, out=out)
        torch.cuda.synchronize()
        if not variant and not np.array_equal(out[:k].cpu().numpy().view(np.uint32), want):
            raise SystemExit(f"hash bench parity check failed (packed, {width}-byte bounds)")
        mv = total + (width + 4) * n
        packed[f"packed_u{8 * width}"] = {
            "api": f"lv_hash_batch_packed, {width}-byte bounds", "value": round(n / (pavg * 1e-3) / 1e9, 3),
            "unit": "Gkeys/s", "ms_avg": round(pavg, 4), "ms_p50": round(pp50, 4), "_ms": pavg,
            "with_metadata": {"bytes_per_launch": mv, "frac_of_8TBps": round(mv / (pavg * 1e-3) / 8e12, 4),
                              "note": f"key bytes + {width} B bound read + 4 B output written per key"}}
        del b
    # every key vs the oracle (untimed), then the CPU baseline
    full = np.zeros(n, dtype=np.uint32)
    host_all = arena.cpu().numpy()
    L.oracle_hash_batch(host_all.ctypes.data, offs.ctypes.data, lens.ctypes.data, None, full.ctypes.data, n)
    H.hash_batch(arena, o, ln, out=out)
    torch.cuda.synchronize()
    if not variant and not np.array_equal(out.cpu().numpy().view(np.uint32), full):
        raise SystemExit("hash bench parity check failed (all keys)")
    del host_all
    cpu = hash_cpu_baseline(arena, offs, lens, args.cpu_seconds) if args.cpu_seconds > 0 else None
    del arena, o, ln, out
    torch.cuda.empty_cache()
    # the VALU side (its own rocprofv3 pass, after this process's timed runs)
    valu, valu_note = measure_hash_valu(args) if args.traffic != "off" else (None, "skipped (--traffic off)")
    vget = (lambda k: valu.get(k)) if isinstance(valu, dict) else (lambda k: None)
    for k, rec in packed.items():
        rec["roofline"], rec["roofline_hbm"], rec["roofline_valu"] = hash_rooflines(
            total, rec.pop("_ms"), vget(k), rec["with_metadata"]["bytes_per_launch"])
    moved = total + 16 * n  # key bytes + off/len + out
    roof, roof_hbm, roof_valu = hash_rooflines(total, avg, vget("offsets"), moved)
    res = {"metric": "batched leveldb hash() + cache shard, device-resident", "unit": "Gkeys/s",
           "keys": n, "key_bytes": total, "value": round(n / (avg * 1e-3) / 1e9, 3), "ms_avg": round(avg, 4),
           "ms_p50": round(p50, 4),
           "roofline": roof, "roofline_hbm": roof_hbm, "roofline_valu": roof_valu,
           "valu_source": valu_note if isinstance(valu, dict) else f"none: {valu_note}",
           "with_metadata": {"bytes_per_launch": moved, "GB_per_s": round(moved / (avg * 1e-3) / 1e9, 1),
                             "frac_of_8TBps": round(moved / (avg * 1e-3) / 8e12, 4),
                             "note": "key bytes + 8 B offset + 4 B length read + 4 B output written per key"},
           "parity": "all keys vs oracle (offsets API), first 100000 keys (every API)", "cpu_baseline": cpu,
           "api": "lv_hash_batch_device (offset + length per key)", **packed,
           "data": "synthetic splitmix64 keys in HBM"}
    print(json.dumps(res), flush=True)
    return res


def parse_cpulist(text):
    """The CPUs of a sysfs cpulist ("0-63,128-191") as a set."""
    cpus = set()
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        cpus.update(range(int(a), int(b or a) + 1))
    return cpus


def confine_to_gpu_socket(device=0):
    """The calling process's CPUs -> the allowed CPUs local to `device` (its
    PCI function's local_cpulist), before it allocates host memory, so the log
    pages, the Reader and the library's copy threads share the GPU's socket:
    the placement a deployment gives a recovery process (numactl
    --cpunodebind).  Returns what was done.  (Round 6, profiles/r06/numa/:
    binding only the library's own threads, with the caller floating, made
    the host paths slower -- the caller's memory decides -- so the placement
    is the caller's, here the bench's.)"""
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, device) != 0:
            return {"placement": "float", "reason": "no PCI bus id"}
        bdf = buf.value.decode().lower()
        text = open(f"/sys/bus/pci/devices/{bdf}/local_cpulist").read().strip()
    except Exception as e:  # noqa: BLE001 - report, never fail the bench on topology
        return {"placement": "float", "reason": f"topology unavailable: {e}"}
    local = parse_cpulist(text)
    allowed = os.sched_getaffinity(0)
    cpus = local & allowed
    if not cpus:
        return {"placement": "float", "reason": "no allowed CPU local to the GPU"}
    os.sched_setaffinity(0, cpus)
    return {"placement": "gpu-local", "gpu_pci": bdf, "cpus": len(cpus), "of_allowed": len(allowed)}


def wal_bench(args):
    """SURVEY 8f rows 1-2 end to end from host memory: group-commit encode
    (lv_wal_encode_host: layout + one GPU CRC batch) and whole-log verify
    (lv_wal_scan_host: H2D, block framing, one CRC batch, D2H), then the host
    Reader over the scan.  Records: logical sizes Random(301).skewed(17)
    (log_writer.rs:456-458, 567), random payload, until ~1 GiB.  The first
    2000 physical records' CRCs are checked against the oracle.  The process
    is first confined to the GPU's socket (--host-placement, default
    gpu-local; confine_to_gpu_socket)."""
    placement = confine_to_gpu_socket() if args.host_placement == "gpu-local" else {"placement": "float"}
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
    # the same Reader loop as a native caller runs it: lv_wal_reader_read_record
    # in one C loop (tools/host_replay.c), no per-record FFI hop
    if lvgpu.experiment_variant() and os.environ.get("LVGPU_LIB"):
        # a timing variant: its lv_* symbols first in the global scope, so the
        # replay helper (linked against the product library) binds to them
        ctypes.CDLL(os.environ["LVGPU_LIB"], mode=os.RTLD_GLOBAL | os.RTLD_NOW)
    R = ctypes.CDLL(os.path.join(ROOT, "leveldb-rs_amd", "lib", "libhostreplay.so"))
    R.lv_replay_reader.restype = ctypes.c_double
    R.lv_replay_reader.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    nr, nb = ctypes.c_uint64(), ctypes.c_uint64()
    t_native = R.lv_replay_reader(out.ctypes.data, out.size, sc._h, 5, ctypes.byref(nr), ctypes.byref(nb))
    if t_native < 0 or nr.value != sizes.size or nb.value != int(sizes.sum()):
        raise SystemExit(f"native reader replay failed: {t_native} s, {nr.value} records, {nb.value} bytes")
    # the recovery pass pipelined: the Reader replays chunk k while the scan of
    # chunk k + 1 runs (lv_wal_scan_host_pipelined), end to end from host memory
    R.lv_replay_recover.restype = ctypes.c_double
    R.lv_replay_recover.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    t_rec = R.lv_replay_recover(out.ctypes.data, out.size, 0, 5, ctypes.byref(nr), ctypes.byref(nb))
    if t_rec < 0 or nr.value != sizes.size or nb.value != int(sizes.sum()):
        raise SystemExit(f"pipelined recovery failed: {t_rec} s, {nr.value} records, {nb.value} bytes")
    # the same recovery with the log in page-locked memory (a caller that read
    # the log file into an lv_host_alloc buffer): the worker DMAs each chunk
    # straight from it, with no staging copy on the CPU beside the Reader
    pin = lvgpu.host_alloc(out.size)
    pin[:] = out
    t_rec_pin = R.lv_replay_recover(pin.ctypes.data, pin.size, 0, 5, ctypes.byref(nr), ctypes.byref(nb))
    if t_rec_pin < 0 or nr.value != sizes.size or nb.value != int(sizes.sum()):
        raise SystemExit(f"pipelined recovery (pinned log) failed: {t_rec_pin} s, {nr.value} records")
    del pin
    # its parts: the pipelined scan alone (to completion), and the Reader over
    # a completed chunked scan
    R.lv_replay_scan_pipelined.restype = ctypes.c_double
    R.lv_replay_scan_pipelined.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
    t_pscan = R.lv_replay_scan_pipelined(out.ctypes.data, out.size, 0, 5)
    psc = LW.Scan.host_pipelined(log)
    psc.wait()
    t_pread = R.lv_replay_reader(out.ctypes.data, out.size, psc._h, 5, ctypes.byref(nr), ctypes.byref(nb))
    del psc
    if t_pscan < 0 or t_pread < 0:
        raise SystemExit(f"pipelined scan parts failed: {t_pscan}, {t_pread}")
    cpu = wal_cpu_baseline(out, args.cpu_seconds, int(o.size)) if args.cpu_seconds > 0 else None
    gib = out.size / 2**30
    print(json.dumps({"metric": "WAL group-commit encode and whole-log verify, host memory end to end",
                      "unit": "GiB/s of log", "log_bytes": int(out.size), "records": int(sizes.size),
                      "physical_records": int(o.size), "host_placement": placement,
                      "encode": {"GiB_per_s": round(gib / t_enc, 2), "ms": round(t_enc * 1e3, 2),
                                 "api": "lv_wal_encode_host"},
                      "scan": {"GiB_per_s": round(gib / t_scan, 2), "ms": round(t_scan * 1e3, 2),
                               "api": "lv_wal_scan_host (H2D + framing + CRC batch + D2H)"},
                      "reader_ms": round(t_read * 1e3, 1),
                      "reader_note": "host Reader replay via ctypes, one call per record (not a GPU figure)",
                      "reader_native": {"ms": round(t_native * 1e3, 2), "GiB_per_s": round(gib / t_native, 2),
                                        "records": int(nr.value),
                                        "note": "lv_wal_reader_read_record in one C loop (tools/host_replay.c), "
                                                "best of 5 whole-log passes over the GPU scan"},
                      "scan_plus_native_reader": {"ms": round((t_scan + t_native) * 1e3, 2),
                                                  "GiB_per_s": round(gib / (t_scan + t_native), 2),
                                                  "note": "whole-log verify from host memory as a native caller "
                                                          "sees it: lv_wal_scan_host then the Reader loop"},
                      "recovery_pipelined": {"ms": round(t_rec * 1e3, 2), "GiB_per_s": round(gib / t_rec, 2),
                                             "records": int(nr.value),
                                             "note": "lv_wal_scan_host_pipelined + the Reader loop + free, one C "
                                                     "loop (tools/host_replay.c), best of 5: the Reader replays "
                                                     "32 MiB chunk k while chunk k + 1 is uploaded and scanned",
                                             "parts_ms": {"pipelined_scan_alone": round(t_pscan * 1e3, 2),
                                                          "reader_over_finished_chunks": round(t_pread * 1e3, 2)}},
                      "recovery_pipelined_pinned_log": {
                          "ms": round(t_rec_pin * 1e3, 2), "GiB_per_s": round(gib / t_rec_pin, 2),
                          "note": "the same recovery over the log in an lv_host_alloc (page-locked) buffer, as a "
                                  "caller that reads the log file into one sees it: chunks DMA'd directly, no CPU "
                                  "staging copy beside the Reader; best of 5"},
                      "cpu_baseline": cpu,
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
    if args.variants:
        return variants_bench(args)
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

    # Timed region (value): K steps between barrier + synchronize, nothing
    # else on the stream, max over ranks of each rank's own time
    # (lvgpu.shard.timed_steps, the code the gloo test drives).  A timestamp
    # event between launches costs ~3 % of the step time on MI355X, so the
    # per-launch HIP events for roofline.achieved are taken in a second pass
    # of the same K steps, right after, on the launch stream.
    head = timed_line(torch, step, stream, args, dist, backend, dev, chunk=20, active=n > 0)
    kern_ms = head["kern_ms"]
    kern_avg_ms = sum(kern_ms) / len(kern_ms)
    own = rank_record(torch, dev, rank, local, nbytes, args.steps, head["timing"], kern_avg_ms)
    if n > 0:  # every rank checks a sample of its own batch against the oracle
        if args.scaling == "weak":
            own["parity_sample"] = rank_sample_check(off, ln, out, n, PAYLOAD_SEED ^ (shard_rank * 0x9E3779B9))
        elif args.workload in ("c3", "c5"):  # a uniform global batch: its global offsets
            own["parity_sample"] = rank_sample_check(off, ln, out, n, None, sh)
    per_rank = shard.gather_ranks(own, dist, world)
    if n > 0 and not all(r.get("parity_sample", True) for r in per_rank):
        raise SystemExit("parity sample failed on rank(s) "
                         + str([r["rank"] for r in per_rank if not r.get("parity_sample", True)]))
    agg = shard.aggregate(per_rank, args.steps, head["timing"].own_max)
    agg_b = shard.aggregate(per_rank, args.steps, head["timing"].barrier_max)
    value = agg["GiB_per_s"]
    achieved_gbs = nbytes / (kern_avg_ms * 1e-3) / 1e9
    kernel = lvgpu.last_kernel()

    # BASELINE configs[4]: one global batch of 64 GiB of
    # 4 KiB blocks split into contiguous rank ranges, timed the same way.  It
    # rides in every default line (N = 1 and the driver's N > 1 lines) as the
    # `c5_strong` sub-record; `value` stays C3 so SCALE N=1 equals BENCH.
    c5 = None
    if c5_wanted(args):
        c5 = c5_strong_record(torch, lvgpu, args, dist, backend, dev, rank, local, world, shard_rank, shard_world)

    # Everything after this point is rank 0's alone and outside every timed
    # region: the other ranks leave the group first, so a slow CPU baseline or
    # PMC pass can never hold them in a collective.
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    result = None
    if rank == 0:
        cpu = None
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
            "world_size": world,
            "launcher": os.environ.get("LVGPU_LAUNCHER", "torch.distributed.run" if world > 1 else "single process"),
            "backend": backend if world > 1 else None,
            "distinct_devices": len({(r["hostname"], r["pci_bus_id"]) for r in per_rank}),
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(agg["ms_per_step"], 4),
            "timing": TIMING_NOTE,
            "value_barrier_inclusive": round(agg_b["GiB_per_s"], 2),
            "ms_per_step_barrier_inclusive": round(agg_b["ms_per_step"], 4),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (splitmix64 payload generated in HBM)",
            "config": {"workload": desc, "buffers_per_gpu": n, "bytes_per_gpu": nbytes,
                       "total_bytes_per_step": agg["total_bytes_per_step"],
                       "api": "lv_crc32c_batch_strided" if strided else "lv_crc32c_batch_device",
                       "parallelism": (f"dp{world} (independent shards, no collective)" if args.scaling == "weak"
                                       else f"dp{world} (one global batch split into contiguous rank ranges, "
                                            f"no collective)")},
            "hbm_peak_frac": round(value * 2**30 / world / 1e9 / HBM_PEAK_GBS, 4),
            "settle": head["settle"],
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
            "c5_strong": c5,
        }
        print(json.dumps(result), flush=True)
    return result


TIMING_NOTE = ("value = bytes of all ranks x steps / max over ranks of each rank's own time (opening barrier + "
               "sync -> K steps -> sync); *_barrier_inclusive: the same up to the end of the closing barrier")


def timed_line(torch, step, stream, args, dist, backend, dev, chunk, active=True):
    """settle -> warmup -> the K timed steps (shard.timed_steps) -> a second
    pass of K steps with a HIP event pair around each launch on `stream`."""
    from lvgpu import shard
    settle_info = settle(torch, step, stream, chunk=chunk) if args.settle and active else None
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    tm = shard.timed_steps(
        step, args.steps, torch.cuda.synchronize, dist,
        lambda x: torch.tensor(x, dtype=torch.float64, device=dev if backend == "nccl" else "cpu"))
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    torch.cuda.synchronize()
    for s, e in evs:
        s.record(stream)
        step()
        e.record(stream)
    torch.cuda.synchronize()
    kern_seq = [s.elapsed_time(e) for s, e in evs]
    if os.environ.get("LVGPU_BENCH_TRACE"):
        print("per-launch ms:", " ".join(f"{x:.4f}" for x in kern_seq), file=sys.stderr)
    return {"settle": settle_info, "timing": tm, "kern_ms": sorted(kern_seq)}


def rank_record(torch, dev, rank, local, nbytes, steps, tm, kern_avg_ms):
    """This rank's entry of `per_gpu` (SURVEY 8e per-GPU figures)."""
    props = torch.cuda.get_device_properties(dev)
    return {"rank": rank, "device": local,
            "pci_bus_id": f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}",
            "gpu_uuid": str(getattr(props, "uuid", "")), "hostname": socket.gethostname(),
            "payload_bytes": nbytes,
            "own_ms_per_step": round(tm.own / steps * 1e3, 4),
            "GiB_per_s": round(nbytes * steps / 2**30 / tm.own, 2),
            "kernel_GB_per_s": round(nbytes / (kern_avg_ms * 1e-3) / 1e9, 1),
            "frac_of_8TBps": round(nbytes / (kern_avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


C5_BLOCKS = 16777216  # BASELINE configs[4]: 64 GiB of 4 KiB blocks


def c5_wanted(args):
    """The C5 sub-record rides in the default line: the C3 weak headline over
    the strided API, not a --as-rank replay (the PMC child) and not asked off."""
    return (args.c5_strong == "auto" and args.workload == "c3" and args.scaling == "weak"
            and args.api == "strided" and args.as_world == 1 and not args.blocks and not args.group)


def c5_strong_record(torch, lvgpu, args, dist, backend, dev, rank, local, world, shard_rank, shard_world):
    """BASELINE configs[4] at this world size: the global batch of C5_BLOCKS x
    4 KiB split by RankShard.uniform, this rank's range generated at its
    byte_lo of the one global splitmix arena, K steps timed like the headline.
    A sample of every rank's blocks (its first and last 8) is checked against
    the oracle over host bytes generated at the same global offsets."""
    from lvgpu import shard
    n_total = C5_BLOCKS
    bl = 4096
    sh = shard.RankShard.uniform(n_total, bl, shard_rank, shard_world)
    arena = torch.empty(max(sh.byte_hi - sh.byte_lo, 1), dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(arena, sh.byte_lo, PAYLOAD_SEED)
    out = torch.empty(max(sh.n, 1), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()

    def step():
        if sh.n:
            lvgpu.batch_strided(arena, bl, bl, sh.n, out=out, stream=stream)
    # one launch is 10.6 ms at N = 1 (1.3 ms at N = 8): settle chunks of ~3 ms
    chunk = max(1, min(20, round(0.003 / max(sh.payload_bytes / 6.5e12, 1e-6))))
    line = timed_line(torch, step, stream, args, dist, backend, dev, chunk=chunk, active=sh.n > 0)
    kern_ms = line["kern_ms"]
    kern_avg = sum(kern_ms) / len(kern_ms)
    rec = rank_record(torch, dev, rank, local, sh.payload_bytes, args.steps, line["timing"], kern_avg)
    rec.update(blocks=[sh.lo, sh.hi], byte_lo=sh.byte_lo, parity_sample=c5_sample_check(arena, out, sh))
    del arena
    per = shard.gather_ranks(rec, dist, world)
    agg = shard.aggregate(per, args.steps, line["timing"].own_max)
    agg_b = shard.aggregate(per, args.steps, line["timing"].barrier_max)
    if not all(r["parity_sample"] for r in per):
        raise SystemExit("c5_strong parity sample failed on rank(s) "
                         + str([r["rank"] for r in per if not r["parity_sample"]]))
    return {"metric": "GiB/s device-resident batched CRC32C, BASELINE configs[4]: 64 GiB of 4 KiB blocks "
                      "sharded across the GPUs (strong scaling)",
            "value": round(agg["GiB_per_s"], 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(agg["ms_per_step"], 4),
            "value_barrier_inclusive": round(agg_b["GiB_per_s"], 2),
            "ms_per_step_barrier_inclusive": round(agg_b["ms_per_step"], 4),
            "scaling": "strong", "timing": TIMING_NOTE,
            "hbm_peak_frac": round(agg["GiB_per_s"] * 2**30 / world / 1e9 / HBM_PEAK_GBS, 4),
            "config": {"workload": f"c5: global batch {n_total} x {bl} B ({n_total * bl / 2**30:.0f} GiB), "
                                   f"RankShard.uniform contiguous rank ranges", "global_buffers": n_total,
                       "global_bytes": n_total * bl, "api": "lv_crc32c_batch_strided",
                       "parallelism": f"dp{world} (one global batch split into contiguous rank ranges, "
                                      f"no collective)"},
            "settle": line["settle"], "rank0_kernel_ms_avg": round(kern_avg, 4),
            "per_gpu": per, "load_imbalance": round(agg["imbalance"], 4),
            "parity": "every rank's first and last 8 blocks vs the oracle over host bytes generated at the "
                      "same global offsets"}


def rank_sample_check(off, ln, out, n, seed, sh=None, k=8):
    """This rank's first and last k buffers vs the oracle over host bytes
    from the oracle's own splitmix generator: at the buffers' offsets in the
    rank's arena (weak scaling: each rank's arena generated from offset 0 with
    its own seed), or -- one global batch (strong) -- at their global offsets."""
    import numpy as np
    if sh is not None:
        return c5_sample_check(None, out, sh, k)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import wal_oracle as W
    L = W.lib()
    got = out[:n].cpu().numpy().view(np.uint32)
    offs = off.cpu().numpy().astype(np.uint64)
    lens = ln.cpu().numpy().view(np.uint32)
    for lo in sorted({0, max(0, n - k)}):
        m = min(k, n - lo)
        o, l = offs[lo:lo + m], lens[lo:lo + m]
        b0 = int(o.min())
        buf = np.empty(max(1, int((o + l).max()) - b0), dtype=np.uint8)
        L.oracle_fill_splitmix(buf.ctypes.data, b0, buf.size, seed)
        ho = (o - np.uint64(b0)).astype(np.uint64)
        hl = np.ascontiguousarray(l, dtype=np.uint32)
        want = np.zeros(m, dtype=np.uint32)
        L.oracle_batch(buf.ctypes.data, ho.ctypes.data, hl.ctypes.data, None, want.ctypes.data, m, 0)
        if not np.array_equal(got[lo:lo + m], want):
            return False
    return True


def c5_sample_check(arena, out, sh, k=8):
    """The rank's first and last k blocks vs the oracle: the host bytes come
    from the oracle's generator at the blocks' GLOBAL byte offsets, so this
    also checks that the range was generated where it belongs in the arena."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import wal_oracle as W
    L = W.lib()
    if sh.n == 0:
        return True
    got = out[:sh.n].cpu().numpy().view(np.uint32)
    for lo in sorted({0, max(0, sh.n - k)}):
        m = min(k, sh.n - lo)
        bl = int(sh.lens[0])
        buf = np.empty(m * bl, dtype=np.uint8)
        L.oracle_fill_splitmix(buf.ctypes.data, sh.byte_lo + lo * bl, buf.size, PAYLOAD_SEED)
        want = np.zeros(m, dtype=np.uint32)
        ho = np.arange(m, dtype=np.uint64) * np.uint64(bl)  # named: the C call reads them
        hl = np.full(m, bl, dtype=np.uint32)
        L.oracle_batch(buf.ctypes.data, ho.ctypes.data, hl.ctypes.data, None, want.ctypes.data, m, 0)
        if not np.array_equal(got[lo:lo + m], want):
            return False
    return True


if __name__ == "__main__":
    main()
