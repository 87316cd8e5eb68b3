"""Phase timeline of wal_pipe_kernel (timing variant LVK_WAL_PIPE_TRACE=1):
per workgroup, s_memrealtime stamps (100 MHz) of its phases, over the bench
log of bench.py --wal-device.  Run with the variant library:

    bash tools/build_variant.sh walptrace -DLVK_WAL_PIPE_TRACE=1
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$PWD/leveldb-rs_amd/lib/variants/liblvgpu_walptrace.so \
        python tools/wal_pipe_trace.py

Prints percentiles over workgroups (us from the earliest start) of: hop 1
sorted, each framer wave done, counts published, look-back done, phase-B list
ready, waves' phase A done / ready seen / walks done, and the end."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leveldb-rs_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import lvgpu  # noqa: E402
import lvgpu.wal as LW  # noqa: E402
import wal_oracle as W  # noqa: E402

KT = 64
r = W.Random(301)
sizes, tot = [], 0
while tot < 262144 * 4096:
    n = r.skewed(17)
    sizes.append(n)
    tot += n
sizes = np.array(sizes, dtype=np.uint64)
payload = np.random.default_rng(7).integers(0, 256, size=int(tot), dtype=np.uint8)
offs = np.zeros(sizes.size, dtype=np.uint64)
offs[1:] = np.cumsum(sizes[:-1])
L = LW._bind()
need = ctypes.c_size_t()
L.lv_wal_encode_host(payload.ctypes.data, offs.ctypes.data, sizes.ctypes.data, sizes.size, 0, None, 0,
                     ctypes.byref(need), 0)
log = np.empty(need.value, dtype=np.uint8)
assert L.lv_wal_encode_host(payload.ctypes.data, offs.ctypes.data, sizes.ctypes.data, sizes.size, 0,
                            log.ctypes.data, log.size, ctypes.byref(need), 0) == 0
d_log = torch.from_numpy(log).to("cuda:0")
LW.set_scan_path(1)  # the one-launch scan (the library's default is the five-launch one)
_, _, _, count = LW.scan_device(d_log, 0)
torch.cuda.synchronize()
cap = int(count.item())
ws = torch.zeros(LW.scan_workspace_bytes(log.size, cap), dtype=torch.uint8, device="cuda:0")
assert ws.numel() >= 16 + 1024 * KT * 8
runs = []
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    hdr, crc, info, cnt = LW.scan_device(d_log, cap, workspace=ws)
    torch.cuda.synchronize()
    assert int(cnt.item()) == cap
    tr = ws[16:16 + 1024 * KT * 8].cpu().numpy().view(np.uint64).reshape(1024, KT).astype(np.int64)
    grid = int((tr[:, 0] != 0).sum())
    tr = tr[:grid]
    t0 = tr[:, 0].min()
    us = (tr - t0) / 100.0  # 100 MHz
    def pct(v):
        v = np.asarray(v, dtype=float)
        return {"p0": round(float(v.min()), 1), "p50": round(float(np.median(v)), 1),
                "p90": round(float(np.percentile(v, 90)), 1), "p100": round(float(v.max()), 1)}
    fr = np.where(tr[:, 3] != 0, np.maximum(us[:, 2], us[:, 3]), us[:, 2])
    runs.append({"grid": grid, "start": pct(us[:, 0]), "hop1_sorted": pct(us[:, 1]), "framed": pct(fr),
                 "published": pct(us[:, 4]), "lookback_done": pct(us[:, 5]), "ready": pct(us[:, 6]),
                 "phaseA_done_first_wave": pct(us[:, 8:24].min(1)), "phaseA_done_last_wave": pct(us[:, 8:24].max(1)),
                 "ready_seen_last_wave": pct(us[:, 24:40].max(1)),
                 "walk_done_first_wave": pct(us[:, 40:56].min(1)), "walk_done_last_wave": pct(us[:, 40:56].max(1)),
                 "end": pct(us[:, 56]),
                 # wave time lost per workgroup, as a fraction of its waves x its end:
                 # waiting for the phase-B list after phase A, and idle after the walk
                 "idle_wait_list": pct(100 * np.clip(us[:, 24:40] - us[:, 8:24], 0, None).sum(1) / (16 * us[:, 56])),
                 "idle_after_walk": pct(100 * (us[:, 56:57] - us[:, 40:56]).sum(1) / (16 * us[:, 56])),
                 "idle_units": "percent of the workgroup's 16 waves x its end"})
    # per-wave stamps of the first-, median- and last-ending workgroups
    order = np.argsort(us[:, 56])
    runs[-1]["waves"] = {name: {"wg": int(order[k]), "framed": round(float(fr[order[k]]), 1),
                                "ready": round(float(us[order[k], 6]), 1),
                                "phaseA_done": [round(float(x), 1) for x in us[order[k], 8:24]],
                                "ready_seen": [round(float(x), 1) for x in us[order[k], 24:40]],
                                "walk_done": [round(float(x), 1) for x in us[order[k], 40:56]],
                                "end": round(float(us[order[k], 56]), 1)}
                         for name, k in (("first", 0), ("median", grid // 2), ("last", grid - 1))}
print(json.dumps(runs[-1], indent=1))
