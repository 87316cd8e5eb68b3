"""Times lv_crc32c_batch_multi on a scattered gather (every range packed on the
host) and, beside it, what round 4's per-call pinning cost: one hipHostMalloc
+ hipHostFree of the pack chunk (256 MiB).  ADVICE r04: the pack buffer is
now cached per device.  Usage: python tools/multi_pack_probe.py [reps]"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "leveldb-rs_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (binds the HIP runtime first)

import lvgpu  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
rng = np.random.default_rng(5)
arena_n = 1 << 30
arena = np.frombuffer(rng.bytes(arena_n), dtype=np.uint8)
n = 32768
lens = rng.integers(1024, 8192, size=n).astype(np.uint32)  # ~150 MiB of payload, shuffled over 1 GiB
offs = rng.integers(0, arena_n - 8192, size=n).astype(np.uint64)
payload = int(lens.sum(dtype=np.uint64))
lvgpu.batch_multi(arena, offs, lens, None, devices=[0])  # warm: contexts, pack buffer
times = []
for _ in range(reps):
    t = time.perf_counter()
    lvgpu.batch_multi(arena, offs, lens, None, devices=[0])
    times.append(time.perf_counter() - t)
hip = ctypes.CDLL("libamdhip64.so")
p = ctypes.c_void_p()
pin = []
for _ in range(reps):
    t = time.perf_counter()
    assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(256 << 20), 0) == 0
    assert hip.hipHostFree(p) == 0
    pin.append(time.perf_counter() - t)
print(json.dumps({"probe": "multi_pack", "payload_bytes": payload, "buffers": n, "reps": reps,
                  "multi_call_ms_median": 1e3 * float(np.median(times)),
                  "multi_GiBps": payload / float(np.median(times)) / 2**30,
                  "pin_alloc_free_256MiB_ms_median": 1e3 * float(np.median(pin)),
                  "note": "round 4 paid the pin line once per packed chunk per call; round 5 pays it once per process"}))
