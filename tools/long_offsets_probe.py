#!/usr/bin/env python3
"""Few long buffers through the offsets API (sort split + class kernel +
combine_long_kernel), for a kernel trace:
    rocprofv3 --kernel-trace --stats -- python3 tools/long_offsets_probe.py [n] [bytes] [ws|lib]
(ws: a caller workspace, lv_crc32c_batch_device_ws; lib: the library's).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "leveldb-rs_amd"))


def main():
    import torch
    import lvgpu
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    bl = int(sys.argv[2]) if len(sys.argv) > 2 else 16 << 20
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    lvgpu.device_init()
    arena = torch.empty(n * bl + 64, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(arena, 0, 0x10)
    o = torch.arange(n, dtype=torch.int64, device=dev) * bl
    ln = torch.full((n,), bl, dtype=torch.int32, device=dev)
    ws = torch.empty(lvgpu.workspace_bytes(n), dtype=torch.uint8, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    lib = len(sys.argv) > 3 and sys.argv[3] == "lib"

    def call():
        if lib:
            lvgpu.batch(arena, o, ln, out=out)
        else:
            lvgpu.batch_ws(arena, o, ln, ws, out=out)

    for _ in range(400):
        call()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(50):
        call()
    en.record()
    torch.cuda.synchronize()
    us = st.elapsed_time(en) * 1e3 / 50
    print(f"{n} x {bl} B: {us:.1f} us per call, {n * bl / us / 1e3:.1f} GB/s ({lvgpu.last_kernel()})")


if __name__ == "__main__":
    main()
