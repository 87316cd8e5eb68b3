"""lvgpu — Python mirror of the reference's `leveldb::util::crc32c` module
(src/util/crc32c.rs) over the C ABI in include/lvgpu/crc32c.h, plus the
batched MI355X entry points.

Names and argument meaning follow the reference:
    value(data) -> int            crc32c.rs:40
    extend(crc, data) -> int      crc32c.rs:42-51
    mask(crc) / unmask(masked)    crc32c.rs:53-63
    extend_sw / extend_hw         crc32c.rs:65-118
The batch functions take torch tensors that already live on the GPU (torch is
used only for device memory and streams) and call the HIP kernels through
ctypes.  There is no CPU fallback: if the shared library or the GPU is
missing they raise.
"""
from __future__ import annotations

import ctypes
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
PRODUCT_LIB = os.path.join(os.path.dirname(_PKG), "lib", "liblvgpu.so")


def _lib_path() -> str:
    """The product library, unless an experiment explicitly selects a variant:
    LVGPU_LIB is honoured only together with LVGPU_EXPERIMENT=1 and only for a
    build under lib/variants/ (tools/build_variant.sh, sanitizer builds), which
    never ships to the GPU box (.gpurunignore)."""
    alt = os.environ.get("LVGPU_LIB")
    if not alt or os.environ.get("LVGPU_EXPERIMENT") != "1":
        return PRODUCT_LIB
    variants = os.path.join(os.path.dirname(_PKG), "lib", "variants")
    if os.path.dirname(os.path.realpath(alt)) != os.path.realpath(variants):
        raise RuntimeError(f"LVGPU_LIB must name a build under {variants}")
    return alt


LIB_PATH = _lib_path()


def experiment_variant() -> bool:
    """True when an experiment variant (tools/build_variant.sh) is loaded
    instead of the product library: timing studies only, CRCs may be wrong."""
    return LIB_PATH != PRODUCT_LIB
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(_PKG)), "include", "lvgpu", "crc32c.h")

MASK = 0x1  # LV_CRC_MASK
GROUP_FLAGS = {None: 0, 1: 0x100, 4: 0x200, 16: 0x300, 64: 0x400}  # LV_CRC_GROUP(g)

# log_format.rs:22-29, 62-66
ZERO, FULL, FIRST, MIDDLE, LAST = 0, 1, 2, 3, 4
BLOCK_SIZE = 32768
HEADER_SIZE = 7


class LvError(RuntimeError):
    pass


_lib = None


def lib() -> ctypes.CDLL:
    """Load liblvgpu.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LvError(f"{LIB_PATH} missing: build it with `make -C leveldb-rs_amd`")
    # One HIP runtime per process: liblvgpu.so needs libamdhip64.so, and the
    # first copy loaded serves every later user of that soname.  Loading torch
    # first binds the library to torch's bundled runtime; loading ours first
    # would hand torch the system runtime, after which torch.cuda reports no
    # device (measured on the MI355X image).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    u8p, u32, u64, sz, vp = ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p
    L.lv_crc32c_value.restype = u32
    L.lv_crc32c_value.argtypes = [u8p, sz]
    for f in ("lv_crc32c_extend", "lv_crc32c_extend_sw", "lv_crc32c_extend_hw"):
        getattr(L, f).restype = u32
        getattr(L, f).argtypes = [u32, u8p, sz]
    for f in ("lv_crc32c_mask", "lv_crc32c_unmask"):
        getattr(L, f).restype = u32
        getattr(L, f).argtypes = [u32]
    L.lv_crc32c_combine.restype = u32
    L.lv_crc32c_combine.argtypes = [u32, u32, u64]
    L.lv_crc32c_batch_device.restype = ctypes.c_int
    L.lv_crc32c_batch_device.argtypes = [vp, vp, vp, vp, vp, sz, u32, vp]
    L.lv_crc32c_workspace_bytes.restype = sz
    L.lv_crc32c_workspace_bytes.argtypes = [sz]
    L.lv_crc32c_batch_device_ws.restype = ctypes.c_int
    L.lv_crc32c_batch_device_ws.argtypes = [vp, vp, vp, vp, vp, sz, u32, vp, sz, vp]
    L.lv_crc32c_batch_strided.restype = ctypes.c_int
    L.lv_crc32c_batch_device_hint.restype = ctypes.c_int
    L.lv_crc32c_batch_device_hint.argtypes = [vp, vp, vp, vp, vp, sz, u32, vp, vp, sz, vp]
    L.lv_crc32c_batch_check.restype = ctypes.c_int
    L.lv_crc32c_batch_check.argtypes = [vp, vp]
    L.lv_crc32c_hint_needs_join.restype = ctypes.c_int
    L.lv_crc32c_hint_needs_join.argtypes = [vp, sz, u32]
    L.lv_crc32c_batch_strided.argtypes = [vp, u64, u32, sz, vp, vp, u32, vp]
    L.lv_crc32c_batch_host.restype = ctypes.c_int
    L.lv_crc32c_batch_host.argtypes = [vp, sz, vp, vp, vp, vp, sz, u32, ctypes.c_int]
    L.lv_crc32c_batch_multi.restype = ctypes.c_int
    L.lv_crc32c_batch_multi.argtypes = [vp, sz, vp, vp, vp, vp, sz, u32, ctypes.c_int]
    L.lv_crc32c_batch_multi_devices.restype = ctypes.c_int
    L.lv_crc32c_batch_multi_devices.argtypes = [vp, sz, vp, vp, vp, vp, sz, u32, vp, ctypes.c_int]
    L.lv_device_init.restype = ctypes.c_int
    L.lv_device_init.argtypes = []
    L.lv_last_error.restype = ctypes.c_char_p
    L.lv_last_error.argtypes = []
    L.lv_version.restype = ctypes.c_char_p
    L.lv_version.argtypes = []
    L.lv_crc32c_last_kernel.restype = ctypes.c_char_p
    L.lv_crc32c_last_kernel.argtypes = []
    L.lv_device_counters.restype = ctypes.c_int
    L.lv_device_counters.argtypes = [ctypes.c_int, vp, sz]
    L.lv_fill_splitmix.restype = ctypes.c_int
    L.lv_fill_splitmix.argtypes = [vp, u64, u64, u64, vp]
    L.lv_host_alloc.restype = vp
    L.lv_host_alloc.argtypes = [sz]
    L.lv_host_free.restype = ctypes.c_int
    L.lv_host_free.argtypes = [vp]
    _lib = L
    return L


def _check(rc: int) -> None:
    if rc != 0:
        raise LvError(f"lvgpu error {rc}: {lib().lv_last_error().decode()}")


def declared_symbols() -> list:
    """Function names declared in include/lvgpu/*.h (crc32c.h, wal.h, ...)."""
    import glob
    import re
    names = []
    for path in sorted(glob.glob(os.path.join(os.path.dirname(HEADER_PATH), "*.h"))):
        with open(path) as f:
            text = f.read()
        names += re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s+\*?\s*(lv_[a-z0-9_]+)\s*\(", text, re.M)
    return names


# ---- scalar drop-ins (crc32c.rs) -------------------------------------------

def value(data) -> int:
    b = bytes(data)
    return lib().lv_crc32c_value(b, len(b))


def extend(crc: int, data) -> int:
    b = bytes(data)
    return lib().lv_crc32c_extend(crc & 0xFFFFFFFF, b, len(b))


def extend_sw(crc: int, data) -> int:
    b = bytes(data)
    return lib().lv_crc32c_extend_sw(crc & 0xFFFFFFFF, b, len(b))


def extend_hw(crc: int, data) -> int:
    b = bytes(data)
    return lib().lv_crc32c_extend_hw(crc & 0xFFFFFFFF, b, len(b))


def mask(crc: int) -> int:
    return lib().lv_crc32c_mask(crc & 0xFFFFFFFF)


def unmask(masked_crc: int) -> int:
    return lib().lv_crc32c_unmask(masked_crc & 0xFFFFFFFF)


def combine(crc_a: int, crc_b: int, len_b: int) -> int:
    """extend(s, A + B) from crc_a = extend(s, A), crc_b = value(B), len_b = len(B)
    (an addition, not in the reference: for callers that split long buffers)."""
    return lib().lv_crc32c_combine(crc_a & 0xFFFFFFFF, crc_b & 0xFFFFFFFF, len_b)


# ---- batch (GPU) -----------------------------------------------------------

def _torch():
    import torch
    return torch


def _stream_ptr(stream):
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def _dev_ptr(t, name):
    if t is None:
        return None
    if not t.is_cuda:
        raise LvError(f"{name} must be a CUDA/HIP tensor")
    if not t.is_contiguous():
        raise LvError(f"{name} must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


def _flags(masked, group):
    if group not in GROUP_FLAGS:
        raise LvError(f"group must be one of {sorted(k for k in GROUP_FLAGS if k)}")
    return (MASK if masked else 0) | GROUP_FLAGS[group]


def batch(arena, off, length, seed=None, out=None, masked=False, stream=None, group=None):
    """Device batch: out[i] = [mask](extend(seed[i] or 0, arena[off[i]:off[i]+length[i]])).

    arena: uint8 CUDA tensor; off: int64 (read as u64); length/seed/out: int32
    or uint32 CUDA tensors (read as u32).  Returns `out` (uint32 bits in an
    int32 tensor when allocated here).  Asynchronous on `stream`.
    """
    torch = _torch()
    n = off.numel()
    if length.numel() != n or (seed is not None and seed.numel() != n):
        raise LvError("off/length/seed size mismatch")
    if off.dtype not in (torch.int64, torch.uint64):
        raise LvError("off must be int64")
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=arena.device)
    _check(lib().lv_crc32c_batch_device(
        _dev_ptr(arena, "arena"), _dev_ptr(off, "off"), _dev_ptr(length, "length"),
        _dev_ptr(seed, "seed"), _dev_ptr(out, "out"), n, _flags(masked, group), _stream_ptr(stream)))
    return out


def workspace_bytes(n: int) -> int:
    """Device workspace lv_crc32c_batch_device_ws needs for n buffers."""
    return int(lib().lv_crc32c_workspace_bytes(n))


def batch_ws(arena, off, length, workspace, seed=None, out=None, masked=False, stream=None):
    """`batch` with a caller-owned uint8 device workspace (graph capture,
    concurrent streams)."""
    torch = _torch()
    n = off.numel()
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=arena.device)
    _check(lib().lv_crc32c_batch_device_ws(
        _dev_ptr(arena, "arena"), _dev_ptr(off, "off"), _dev_ptr(length, "length"),
        _dev_ptr(seed, "seed"), _dev_ptr(out, "out"), n, _flags(masked, None),
        _dev_ptr(workspace, "workspace"), workspace.numel(), _stream_ptr(stream)))
    return out


class BatchHint(ctypes.Structure):
    """lv_batch_hint (include/lvgpu/crc32c.h): host-side facts about a batch."""
    _fields_ = [("total_bytes", ctypes.c_uint64), ("max_len", ctypes.c_uint32), ("uniform", ctypes.c_uint32)]


HINT_UNIFORM = 1     # LV_HINT_UNIFORM
HINT_ALIGNED16 = 2   # LV_HINT_ALIGNED16


def hint_for(lengths, offsets=None) -> BatchHint:
    """The exact hint of a host-side length list (numpy-convertible); with the
    host-side offsets too, a uniform batch whose offsets are all multiples of
    16 also gets LV_HINT_ALIGNED16 (the library checks the arena's own
    alignment)."""
    import numpy as np
    ln = np.asarray(lengths, dtype=np.uint64)
    mx = int(ln.max()) if ln.size else 0
    uniform = int(ln.size > 0 and bool((ln == mx).all()))
    if uniform and offsets is not None and bool((np.asarray(offsets, dtype=np.uint64) % 16 == 0).all()):
        uniform |= HINT_ALIGNED16
    return BatchHint(int(ln.sum()), mx, uniform)


def batch_hint(arena, off, length, hint: BatchHint, seed=None, out=None, masked=False, workspace=None,
               stream=None):
    """`batch` with host-side facts about the lengths (lv_crc32c_batch_device_hint):
    the library leaves out launches they prove empty.  `hint` must be exact."""
    torch = _torch()
    n = off.numel()
    if length.numel() != n or (seed is not None and seed.numel() != n):
        raise LvError("off/length/seed size mismatch")
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=arena.device)
    _check(lib().lv_crc32c_batch_device_hint(
        _dev_ptr(arena, "arena"), _dev_ptr(off, "off"), _dev_ptr(length, "length"),
        _dev_ptr(seed, "seed"), _dev_ptr(out, "out"), n, _flags(masked, None),
        ctypes.byref(hint) if hint is not None else None, _dev_ptr(workspace, "workspace"),
        workspace.numel() if workspace is not None else 0, _stream_ptr(stream)))
    return out


HINT_ERR_MISALIGNED = 0x1   # LV_HINT_ERR_MISALIGNED
HINT_ERR_NOT_UNIFORM = 0x2  # LV_HINT_ERR_NOT_UNIFORM
HINT_ERR_LONGER = 0x4       # LV_HINT_ERR_LONGER
HINT_ERR_TOTAL = 0x8        # LV_HINT_ERR_TOTAL
ERR_HINT = -4               # LV_ERR_HINT


class HintViolation(LvError):
    """A batch hint contradicted the device-side offsets/lengths
    (lv_crc32c_batch_check); `violations` holds the LV_HINT_ERR_* bits."""

    def __init__(self, msg, violations):
        super().__init__(msg)
        self.violations = violations


def batch_check(stream=None) -> None:
    """Wait for `stream` and raise HintViolation if a hinted batch call on it
    (since the last check) was given facts its device arrays contradict."""
    v = ctypes.c_uint32(0)
    rc = lib().lv_crc32c_batch_check(_stream_ptr(stream), ctypes.byref(v))
    if rc == ERR_HINT:
        raise HintViolation(f"lvgpu error {rc}: {lib().lv_last_error().decode()}", int(v.value))
    _check(rc)


def batch_strided(base, stride: int, block_len: int, n: int, seed=None, out=None, masked=False, stream=None,
                  group=None):
    """Device batch over n fixed-size blocks base[i*stride : i*stride+block_len]."""
    torch = _torch()
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=base.device)
    if n and (n - 1) * stride + block_len > base.numel():
        raise LvError("blocks exceed base tensor")
    _check(lib().lv_crc32c_batch_strided(
        _dev_ptr(base, "base"), stride, block_len, n, _dev_ptr(seed, "seed"), _dev_ptr(out, "out"),
        _flags(masked, group), _stream_ptr(stream)))
    return out


def batch_host(arena: bytes, off, length, seed=None, masked=False, device: int = 0):
    """Host-memory batch (pinned staging + H2D + kernel + D2H, synchronous).
    off/length/seed are numpy arrays (uint64 / uint32); returns np.uint32 array."""
    import numpy as np
    a = np.frombuffer(arena, dtype=np.uint8) if isinstance(arena, (bytes, bytearray)) else np.ascontiguousarray(arena, dtype=np.uint8)
    o = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(length, dtype=np.uint32)
    sd = None if seed is None else np.ascontiguousarray(seed, dtype=np.uint32)
    n = o.size
    out = np.empty(n, dtype=np.uint32)
    _check(lib().lv_crc32c_batch_host(
        a.ctypes.data_as(ctypes.c_void_p), a.size, o.ctypes.data_as(ctypes.c_void_p),
        ln.ctypes.data_as(ctypes.c_void_p), None if sd is None else sd.ctypes.data_as(ctypes.c_void_p),
        out.ctypes.data_as(ctypes.c_void_p), n, MASK if masked else 0, device))
    return out


def batch_multi(arena: bytes, off, length, seed=None, masked=False, ngpu: int = None, devices=None):
    """Host-memory batch split by payload bytes over devices 0..ngpu-1 (or an
    explicit `devices` list, repeats allowed); returns np.uint32 array."""
    import numpy as np
    a = np.frombuffer(arena, dtype=np.uint8) if isinstance(arena, (bytes, bytearray)) else np.ascontiguousarray(arena, dtype=np.uint8)
    o = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(length, dtype=np.uint32)
    sd = None if seed is None else np.ascontiguousarray(seed, dtype=np.uint32)
    out = np.empty(o.size, dtype=np.uint32)
    vp = ctypes.c_void_p
    args = (a.ctypes.data_as(vp), a.size, o.ctypes.data_as(vp), ln.ctypes.data_as(vp),
            None if sd is None else sd.ctypes.data_as(vp), out.ctypes.data_as(vp), o.size, MASK if masked else 0)
    if devices is not None:
        d = np.ascontiguousarray(devices, dtype=np.int32)
        _check(lib().lv_crc32c_batch_multi_devices(*args, d.ctypes.data_as(vp), d.size))
    else:
        _check(lib().lv_crc32c_batch_multi(*args, 1 if ngpu is None else ngpu))
    return out


def host_alloc(nbytes: int):
    """A page-locked host buffer (lv_host_alloc) as a numpy uint8 array, freed
    (lv_host_free) when the array is released: read a log or table file into
    it and the host entry points DMA it without a staging copy."""
    import weakref

    import numpy as np
    L = lib()
    p = L.lv_host_alloc(nbytes)
    if not p:
        raise LvError(f"lv_host_alloc({nbytes}): {L.lv_last_error().decode()}")
    buf = (ctypes.c_uint8 * max(nbytes, 1)).from_address(p)
    weakref.finalize(buf, L.lv_host_free, p)
    return np.ctypeslib.as_array(buf)[:nbytes]


def fill_splitmix(dst, begin: int, seed: int, stream=None):
    """Fill a uint8 CUDA tensor with the synthetic payload bytes [begin, begin+numel)."""
    _check(lib().lv_fill_splitmix(_dev_ptr(dst, "dst"), begin, dst.numel(), seed, _stream_ptr(stream)))
    return dst


def device_init() -> None:
    _check(lib().lv_device_init())


def version() -> str:
    return lib().lv_version().decode()


def last_kernel() -> str:
    """Kernel the calling thread's last batch call launched (debug query)."""
    return lib().lv_crc32c_last_kernel().decode()


def device_counters(device: int = 0) -> dict:
    """What the host entry points have copied / allocated on `device` so far
    (lv_device_counters): {"h2d": bytes, "d2h": bytes, "allocs": count}."""
    v = (ctypes.c_uint64 * 3)()
    _check(lib().lv_device_counters(device, ctypes.cast(v, ctypes.c_void_p), 3))
    return {"h2d": int(v[0]), "d2h": int(v[1]), "allocs": int(v[2])}
