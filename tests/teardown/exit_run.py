"""Subprocess body of tests/test_teardown.py: loads the HIP interposer
(argv[1]) into the global scope before liblvgpu.so, uses the library (argv[2]:
"bad" -- the negative control; "cpu" -- only lv_host_alloc / lv_host_free, which reach hipHostMalloc /
hipHostFree even without a device; "gpu" -- the host paths that leave
library-owned streams, events, pinned staging and device buffers alive until
exit), arms the interposer in a Python atexit hook and exits normally."""
import atexit
import ctypes
import os
import sys

try:
    import torch  # noqa: F401  (the HIP runtime liblvgpu.so binds to, loaded first as lvgpu.lib() does)
except ImportError:
    pass
spy = ctypes.CDLL(sys.argv[1], mode=os.RTLD_GLOBAL | os.RTLD_NOW)
if sys.argv[2] == "bad":  # negative control: argv[3] is tests/teardown/bad_static.cc built as liblvgpu_*.so
    ctypes.CDLL(sys.argv[3]).lvgpu_bad_probe()
    print("positive_control", spy.hipspy_calls(), flush=True)
    atexit.register(spy.hipspy_arm)
    sys.exit(0)
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "leveldb-rs_amd"))
import lvgpu  # noqa: E402

L = lvgpu.lib()
p = L.lv_host_alloc(4096)
L.lv_host_free(p)
if sys.argv[2] == "gpu":
    import numpy as np

    import lvgpu.wal as LW
    rng = np.random.default_rng(3)
    arena = rng.integers(0, 256, size=1 << 20, dtype=np.uint8).tobytes()
    off = np.arange(256, dtype=np.uint64) * 4096
    out = lvgpu.batch_host(arena, off, np.full(256, 4096, dtype=np.uint32))
    assert int(out[0]) == lvgpu.value(arena[:4096])
    log = LW.encode([arena[i * 3000:(i + 1) * 3000] for i in range(100)])
    r = LW.Reader(log, LW.Scan.host_pipelined(log))
    assert r.read_record() == arena[:3000]
print("positive_control", spy.hipspy_calls(), flush=True)
atexit.register(spy.hipspy_arm)
