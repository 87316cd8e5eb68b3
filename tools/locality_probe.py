#!/usr/bin/env python3
"""Does address locality of the buffers in flight matter to the offsets API?
262,144 x 4 KiB buffers of one 1 GiB arena, listed in address order and in a
random permutation (same lengths, so the same single sort key): the class
kernel then streams adjacent buffers, or buffers scattered over the arena.
    python tools/locality_probe.py
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
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    lvgpu.device_init()
    n, bl = 262144, 4096
    arena = torch.empty(n * bl, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(arena, 0, 0x4C4F43)
    ln = torch.full((n,), bl, dtype=torch.int32, device=dev)
    ws = torch.empty(lvgpu.workspace_bytes(n), dtype=torch.uint8, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    rng = np.random.default_rng(3)
    res = {}
    for name, idx in (("address order", np.arange(n)), ("permuted", rng.permutation(n)),
                      ("permuted in 64 MiB windows", np.concatenate(
                          [w0 + rng.permutation(16384) for w0 in range(0, n, 16384)]))):
        o = torch.from_numpy((idx.astype(np.int64) * bl)).to(dev)
        _, avg = bench._event_times(torch, lambda: lvgpu.batch_ws(arena, o, ln, ws, out=out), 100, 30)
        res[name] = {"ms": round(avg, 4), "frac_of_8TBps": round(n * bl / (avg * 1e-3) / 8e12, 4)}
        print(name, res[name], flush=True)
    print(json.dumps({"probe": "offsets API address locality, 262,144 x 4 KiB", "results": res}))


if __name__ == "__main__":
    main()
