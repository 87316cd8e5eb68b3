"""Round 6 (final): does replaying the C3 headline's launches from a HIP
graph shorten the gap between back-to-back kernels?  262,144 x 4 KiB blocks
through lv_crc32c_batch_strided: 200 launches on a stream against a graph of
20 launches replayed 10 times, three interleaved reps, outputs compared."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "leveldb-rs_amd"))
import lvgpu  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    lvgpu.device_init()
    n = 262144
    arena = torch.empty(n * 4096, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(arena, 0, 0x1234)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream()
    step = lambda: lvgpu.batch_strided(arena, 4096, 4096, n, out=out, stream=s)  # noqa: E731
    with torch.cuda.stream(s):
        for _ in range(50):
            step()
        torch.cuda.synchronize()
        ref = out.clone()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(20):
                step()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, ref), "graph replay output differs"
        res = {"eager_us": [], "graph_us": []}
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(200):
                step()
            e1.record(s)
            torch.cuda.synchronize()
            res["eager_us"].append(round(e0.elapsed_time(e1) * 1e3 / 200, 2))
            e0.record(s)
            for _ in range(10):
                g.replay()
            e1.record(s)
            torch.cuda.synchronize()
            res["graph_us"].append(round(e0.elapsed_time(e1) * 1e3 / 200, 2))
    res["bytes"] = n * 4096
    res["eager_frac"] = [round(n * 4096 / (u * 1e-6) / 8e12, 4) for u in res["eager_us"]]
    res["graph_frac"] = [round(n * 4096 / (u * 1e-6) / 8e12, 4) for u in res["graph_us"]]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
