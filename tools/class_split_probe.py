"""Where does the class kernel spend a mixed batch's time?  Times the offsets
API on a bench workload (c2 / c4) whole and split by length class -- the
same arena, only the buffers of classes {0, 1} (<= 2 KiB) or of classes
{2, 3} -- and prints each subset's bytes, time and fraction of 8 TB/s.
Not a parity test (tests/ hold those); a diagnostic for DESIGN §10.
usage: python3 tools/class_split_probe.py [c2|c4] [steps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "leveldb-rs_amd"))


def main():
    import numpy as np
    import torch
    import lvgpu
    import bench
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    lvgpu.device_init()
    arena, off, ln, total, desc = bench.build_workload(torch, lvgpu, name, dev, 0)
    lens = ln.cpu().numpy().view(np.uint32)
    rows = []
    for tag, mask in (("all", np.ones(lens.size, dtype=bool)), ("small (<= 2 KiB)", lens <= 2048),
                      ("large (> 2 KiB)", lens > 2048), ("class 0 (<= 256 B)", lens <= 256),
                      ("class 1", (lens > 256) & (lens <= 2048)), ("class 2", (lens > 2048) & (lens <= 32768)),
                      ("class 3", lens > 32768)):
        idx = torch.from_numpy(np.nonzero(mask)[0]).to(dev)
        if idx.numel() == 0:
            continue
        o, l = off[idx].contiguous(), ln[idx].contiguous()
        n = int(idx.numel())
        ws = torch.empty(lvgpu.workspace_bytes(n), dtype=torch.uint8, device=dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        fn = lambda: lvgpu.batch_ws(arena, o, l, ws, out=out)
        _, avg = bench._event_times(torch, fn, steps, 20)
        nbytes = int(lens[mask].astype(np.int64).sum())
        rows.append({"subset": tag, "buffers": n, "bytes": nbytes, "us": round(avg * 1e3, 1),
                     "frac_of_8TBps": round(nbytes / (avg * 1e-3) / 8e12, 4), "kernels": lvgpu.last_kernel()})
        print(json.dumps(rows[-1]), flush=True)
    print(json.dumps({"workload": desc, "rows": rows}))


if __name__ == "__main__":
    main()
