import sys, time, numpy as np
sys.path.insert(0, "leveldb-rs_amd"); sys.path.insert(0, "oracle")
import lvgpu, wal_oracle as W
lvgpu.device_init()
rng = np.random.default_rng(3)
a = rng.integers(0, 256, size=(1 << 30) + 64, dtype=np.uint8)
off = np.array([3], dtype=np.uint64); ln = np.array([1 << 30], dtype=np.uint32)
lvgpu.batch_host(a, off, ln)
ts = []
for _ in range(5):
    t0 = time.perf_counter(); got = lvgpu.batch_host(a, off, ln); ts.append(time.perf_counter() - t0)
want = np.zeros(1, dtype=np.uint32)
W.lib().oracle_batch(a.ctypes.data, off.ctypes.data, ln.ctypes.data, None, want.ctypes.data, 1, 0)
print("single 1 GiB buffer via lv_crc32c_batch_host: %.1f ms median, %.1f GiB/s, match=%s" % (sorted(ts)[2] * 1e3, 1 / sorted(ts)[2], bool(got[0] == want[0])))
