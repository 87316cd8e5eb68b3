"""Latency of small strided batches (8-64 KiB blocks, 1-64 MiB per call):
the blocks kernel's staggered start must not delay calls with little work."""
import sys
sys.path.insert(0, "leveldb-rs_amd")
import torch, lvgpu
dev = torch.device("cuda:0"); torch.cuda.set_device(dev); lvgpu.device_init()
arena = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
lvgpu.fill_splitmix(arena, 0, 7)
for kib in (8, 64):
    bl = kib << 10
    for mib in (1, 8, 64):
        n = (mib << 20) // bl
        out = torch.empty(n, dtype=torch.int32, device=dev)
        for _ in range(50): lvgpu.batch_strided(arena, bl, bl, n, out=out)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(100): lvgpu.batch_strided(arena, bl, bl, n, out=out)
        b.record(); torch.cuda.synchronize()
        print(f"{kib} KiB x {n}: {a.elapsed_time(b) / 100 * 1e3:.1f} us", flush=True)
