"""Python mirror of util::hash (src/util/hash.rs:20-51) and the cache shard
choice (src/util/cache.rs:394-399) over include/lvgpu/hash.h."""
from __future__ import annotations

import ctypes

from . import LvError, _check, _dev_ptr, _stream_ptr, _torch, lib

SHARD = 0x1  # LV_HASH_SHARD
_bound = False


def _bind():
    global _bound
    L = lib()
    if not _bound:
        vp, sz, u32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32
        L.lv_hash.restype = u32
        L.lv_hash.argtypes = [ctypes.c_char_p, sz, u32]
        L.lv_cache_shard.restype = u32
        L.lv_cache_shard.argtypes = [u32]
        L.lv_hash_batch_device.restype = ctypes.c_int
        L.lv_hash_batch_device.argtypes = [vp, vp, vp, vp, vp, sz, u32, vp]
        L.lv_hash_batch_packed.restype = ctypes.c_int
        L.lv_hash_batch_packed.argtypes = [vp, vp, u32, vp, vp, sz, u32, vp]
        _bound = True
    return L


def hash(data, seed: int) -> int:  # noqa: A001 — the reference's name
    b = bytes(data)
    return int(_bind().lv_hash(b, len(b), seed & 0xFFFFFFFF))


def cache_shard(h: int) -> int:
    return int(_bind().lv_cache_shard(h & 0xFFFFFFFF))


def hash_batch(arena, off, length, seed=None, out=None, shard=False, stream=None):
    """Device batch: out[i] = hash(arena[off[i]:off[i]+length[i]], seed[i] or 0),
    or its cache shard with shard=True.  Tensors as for lvgpu.batch."""
    torch = _torch()
    L = _bind()
    n = off.numel()
    if length.numel() != n or (seed is not None and seed.numel() != n):
        raise LvError("off/length/seed size mismatch")
    if off.dtype not in (torch.int64, torch.uint64):
        raise LvError("off must be int64")
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=arena.device)
    _check(L.lv_hash_batch_device(_dev_ptr(arena, "arena"), _dev_ptr(off, "off"), _dev_ptr(length, "length"),
                                  _dev_ptr(seed, "seed"), _dev_ptr(out, "out"), n, SHARD if shard else 0,
                                  _stream_ptr(stream)))
    return out


def hash_batch_packed(arena, bounds, seed=None, out=None, shard=False, stream=None):
    """Packed keys: key i = arena[bounds[i]:bounds[i+1]] for n + 1 bounds
    (an int32/uint32 tensor: 4-byte bounds, int64/uint64: 8-byte), as
    lv_hash_batch_packed.  Returns the n hashes (or shards)."""
    torch = _torch()
    L = _bind()
    n = bounds.numel() - 1
    if n < 0:
        raise LvError("bounds needs n + 1 entries")
    width = bounds.element_size()
    if width not in (4, 8):
        raise LvError("bounds must be 4- or 8-byte integers")
    if seed is not None and seed.numel() != n:
        raise LvError("seed size mismatch")
    if out is None:
        out = torch.empty(max(n, 0), dtype=torch.int32, device=arena.device)
    _check(L.lv_hash_batch_packed(_dev_ptr(arena, "arena"), _dev_ptr(bounds, "bounds"), width,
                                  _dev_ptr(seed, "seed"), _dev_ptr(out, "out"), n, SHARD if shard else 0,
                                  _stream_ptr(stream)))
    return out
