"""Strided-API rate for power-of-two block sizes with and without stride
padding (is the 8/16 KiB dip an HBM address-mapping effect?)."""
import json, sys
sys.path.insert(0, "leveldb-rs_amd")
import torch, lvgpu
dev = torch.device("cuda:0"); torch.cuda.set_device(dev); lvgpu.device_init()
total = 2 << 30
arena = torch.empty(total + (1 << 24), dtype=torch.uint8, device=dev)
lvgpu.fill_splitmix(arena, 0, 7)
res = []
for kib in (4, 8, 16, 32):
    bl = kib << 10
    for pad in (0, 256, 4096):
        stride = bl + pad
        n = total // stride
        out = torch.empty(n, dtype=torch.int32, device=dev)
        for _ in range(40): lvgpu.batch_strided(arena, stride, bl, n, out=out)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(50): lvgpu.batch_strided(arena, stride, bl, n, out=out)
        b.record(); torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 50
        res.append((kib, pad, round(n * bl / (ms * 1e-3) / 8e12, 4)))
        print(kib, pad, res[-1][2], flush=True)
