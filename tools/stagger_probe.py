"""Strided-API rate per block size under library variants (LVGPU_LIB set by
the caller): does a staggered wave start change the 8/16 KiB dips?"""
import json, os, sys
sys.path.insert(0, "leveldb-rs_amd")
import torch, lvgpu
dev = torch.device("cuda:0"); torch.cuda.set_device(dev); lvgpu.device_init()
total = 2 << 30
arena = torch.empty(total, dtype=torch.uint8, device=dev)
lvgpu.fill_splitmix(arena, 0, 7)
res = []
for kib in (4, 8, 16, 32, 64):
    bl = kib << 10
    n = total // bl
    out = torch.empty(n, dtype=torch.int32, device=dev)
    for _ in range(40): lvgpu.batch_strided(arena, bl, bl, n, out=out)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(60): lvgpu.batch_strided(arena, bl, bl, n, out=out)
    b.record(); torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 60
    res.append(round(n * bl / (ms * 1e-3) / 8e12, 4))
print(os.path.basename(os.environ.get("LVGPU_LIB", "default")), res, flush=True)
