#!/usr/bin/env python3
"""Where does the SST trailer kernel's time go?  Times lv_sst_verify_blocks_device
(one launch, lvk::sst_blocks_kernel) on ~1 GiB tables of different block-size
shapes, each block followed by its 5-byte trailer (so block starts are
byte-packed, i.e. misaligned), and reports GB/s of contents + type and the
256-B rows the walk loads per block (4-row batches on the absolute 256-B grid).

    python tools/table_shape_probe.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "leveldb-rs_amd"))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    import lvgpu
    import lvgpu.table as T
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    lvgpu.device_init()
    rng = np.random.default_rng(5)
    n = 262144
    shapes = {
        "4096+U[0,256) (bench)": 4096 + rng.integers(0, 256, n),
        "4096 fixed": np.full(n, 4096),
        "4091 fixed (unit 4092, 16 rows)": np.full(n, 4091),
        "3835 fixed (unit 3836, <= 16 rows)": np.full(n, 3835),
        "4352 fixed": np.full(n, 4352),
        "4607 fixed (unit 4608, 18-19 rows)": np.full(n, 4607),
    }
    out = []
    for name, sizes in shapes.items():
        sizes = sizes.astype(np.int64)
        offs = np.zeros(n, dtype=np.int64)
        offs[1:] = np.cumsum(sizes[:-1] + 5)
        total = int(offs[-1] + sizes[-1] + 5)
        f = torch.empty(total, dtype=torch.uint8, device=dev)
        lvgpu.fill_splitmix(f, 0, 0x4C444231)
        h = torch.from_numpy(np.stack([offs, sizes], axis=1).copy()).to(dev)
        T.seal_blocks(f, h)
        p50, avg = bench._event_times(torch, lambda: T.verify_blocks(f, h), 100, 30)
        st = T.verify_blocks(f, h)
        torch.cuda.synchronize()
        assert bool((st == 0).all())
        unit = int(sizes.sum()) + n
        starts = (offs % 256)
        rows = ((starts + sizes + 1 + 255) // 256).mean()
        r = {"shape": name, "GB_per_s": round(unit / (avg * 1e-3) / 1e9, 1),
             "frac_of_8TBps": round(unit / (avg * 1e-3) / 8e12, 4), "ms_avg": round(avg, 4),
             "rows_per_block_mean": round(float(rows), 3),
             "batches_per_block_mean": round(float(np.ceil(((starts + sizes + 1 + 255) // 256) / 4).mean()), 3)}
        print(json.dumps(r), flush=True)
        out.append(r)
        del f, h
    print(json.dumps({"probe": "table shapes", "results": out}))


if __name__ == "__main__":
    main()
