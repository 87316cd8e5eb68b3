"""Host-memory WAL paths under repetition (for the ASan build of the host
code, tools/r05_asan.sh): lv_wal_scan_host_pipelined + the Reader, the
finished scan's flat arrays, lv_wal_scan_host, over logs of 0.1-300 MB,
intact and corrupted, every result checked against lv_wal_scan_host's.
Usage: python tools/pipe_stress.py [iterations]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leveldb-rs_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (binds the HIP runtime first)

import lvgpu.wal as LW  # noqa: E402
import wal_oracle as W  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 12
rng = np.random.default_rng(77)
for it in range(iters):
    n = int(rng.integers(10, 3000 if it % 3 else 30000))
    recs = [rng.integers(0, 256, size=int(rng.integers(0, 1 << int(rng.integers(0, 17)))), dtype=np.uint8).tobytes()
            for _ in range(n)]
    log = bytearray(LW.encode(recs))
    if it % 4 == 3:
        for pos in rng.integers(0, len(log), size=20):
            log[int(pos)] ^= 0x5A
    log = bytes(log)
    a = LW.Scan.host(log)
    b = LW.Scan.host_pipelined(log)
    rep = W.ReportCollector()
    rd = LW.Reader(log, b, rep)
    k = 0
    while rd.read_record() is not None:
        k += 1
    b.wait()
    assert np.array_equal(a.offsets, b.offsets) and np.array_equal(a.crcs, b.crcs) and np.array_equal(a.info, b.info)
    del rd, a, b
    print(f"iter {it}: {len(log)} B, {n} records, {k} read", flush=True)
print("stress ok")
