"""Exit-time probe: uses the library's host paths, which
create library-owned streams, events and pinned buffers that live until the
process exits (lv_crc32c_batch_host: the device's host-path stream and two
events; lv_wal_scan_host_pipelined: a second stream), then returns normally.
Run under `rocprofv3 --kernel-trace --stats` to see whether the process
survives the runtime's teardown with those objects still alive.
usage: python tools/r06/exit_probe.py [host|pipe|device]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "leveldb-rs_amd"))
import lvgpu  # noqa: E402
import lvgpu.wal as LW  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "host"
rng = np.random.default_rng(1)
arena = rng.integers(0, 256, size=1 << 20, dtype=np.uint8).tobytes()
off = np.arange(256, dtype=np.uint64) * 4096
ln = np.full(256, 4096, dtype=np.uint32)
if what in ("host", "pipe"):
    out = lvgpu.batch_host(arena, off, ln)
    assert int(out[0]) == lvgpu.value(arena[:4096])
if what == "pipe":
    log = LW.encode([arena[i * 5000:(i + 1) * 5000] for i in range(150)])
    s = LW.Scan.host_pipelined(log)
    s.wait()
    r = LW.Reader(log, s)
    n = 0
    while r.read_record() is not None:
        n += 1
    assert n == 150, n
if what == "device":
    import torch
    t = torch.frombuffer(bytearray(arena), dtype=torch.uint8).to("cuda:0")
    o = lvgpu.batch_strided(t, 4096, 4096, 256)
    torch.cuda.synchronize()
    assert int(o[0].item()) & 0xffffffff == lvgpu.value(arena[:4096])
print("exit_probe", what, "done", flush=True)
