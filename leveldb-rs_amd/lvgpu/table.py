"""Python mirror of src/table/format.rs (BlockHandle, Footer) and the GPU
block-trailer seal/verify over include/lvgpu/table.h."""
from __future__ import annotations

import ctypes

import numpy as np

from . import LvError, _check, _dev_ptr, _stream_ptr, _torch, lib

MAGIC = 0xDB4775248B80FB57
BLOCK_HANDLE_MAX_ENCODED_LENGTH = 20
FOOTER_ENCODED_LENGTH = 48
TRAILER_SIZE = 5
BLOCK_OK, BLOCK_CHECKSUM_MISMATCH, BLOCK_OUT_OF_RANGE = 0, 1, 2
ERR_CORRUPTION = -3
_bound = False


class Corruption(LvError):
    """ErrorType::Corruption from the format decoders."""


def _bind():
    global _bound
    L = lib()
    if not _bound:
        vp, sz, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64
        L.lv_sst_block_handle_encode.restype = sz
        L.lv_sst_block_handle_encode.argtypes = [u64, u64, ctypes.c_char_p]
        L.lv_sst_block_handle_decode.restype = ctypes.c_int
        L.lv_sst_block_handle_decode.argtypes = [ctypes.c_char_p, sz, ctypes.POINTER(u64), ctypes.POINTER(u64),
                                                 ctypes.POINTER(sz)]
        L.lv_sst_footer_encode.restype = None
        L.lv_sst_footer_encode.argtypes = [u64, u64, u64, u64, ctypes.c_char_p]
        L.lv_sst_footer_decode.restype = ctypes.c_int
        L.lv_sst_footer_decode.argtypes = [ctypes.c_char_p, sz, ctypes.POINTER(u64 * 4)]
        L.lv_sst_seal_blocks_device.restype = ctypes.c_int
        L.lv_sst_seal_blocks_device.argtypes = [vp, u64, vp, vp, sz, vp]
        L.lv_sst_verify_blocks_device.restype = ctypes.c_int
        L.lv_sst_verify_blocks_device.argtypes = [vp, u64, vp, sz, vp, vp, vp]
        L.lv_sst_verify_blocks_host.restype = ctypes.c_int
        L.lv_sst_verify_blocks_host.argtypes = [vp, u64, vp, sz, vp, ctypes.c_int]
        _bound = True
    return L


def _decode_check(rc, L):
    if rc == ERR_CORRUPTION:
        raise Corruption(L.lv_last_error().decode())
    _check(rc)


class BlockHandle:  # format.rs:26-50
    def __init__(self, offset: int, size: int):
        self.offset, self.size = offset, size

    def __eq__(self, o):
        return (self.offset, self.size) == (o.offset, o.size)

    def __repr__(self):
        return f"BlockHandle(offset={self.offset}, size={self.size})"

    def encode_to(self, dst: bytearray) -> None:
        buf = ctypes.create_string_buffer(BLOCK_HANDLE_MAX_ENCODED_LENGTH)
        n = _bind().lv_sst_block_handle_encode(self.offset, self.size, buf)
        dst += buf.raw[:n]

    @staticmethod
    def decode_from(src: bytes):
        """-> (BlockHandle, bytes consumed); Corruption("bad handle")."""
        L = _bind()
        o, s, n = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_size_t()
        b = bytes(src)
        _decode_check(L.lv_sst_block_handle_decode(b, len(b), ctypes.byref(o), ctypes.byref(s), ctypes.byref(n)), L)
        return BlockHandle(o.value, s.value), n.value


class Footer:  # format.rs:52-104
    def __init__(self, metaindex_handle: BlockHandle, index_handle: BlockHandle):
        self.metaindex_handle, self.index_handle = metaindex_handle, index_handle

    def __eq__(self, o):
        return (self.metaindex_handle, self.index_handle) == (o.metaindex_handle, o.index_handle)

    def encode(self) -> bytes:
        out = ctypes.create_string_buffer(FOOTER_ENCODED_LENGTH)
        m, i = self.metaindex_handle, self.index_handle
        _bind().lv_sst_footer_encode(m.offset, m.size, i.offset, i.size, out)
        return out.raw

    @staticmethod
    def decode_from(src: bytes) -> "Footer":
        L = _bind()
        h = (ctypes.c_uint64 * 4)()
        b = bytes(src)
        _decode_check(L.lv_sst_footer_decode(b, len(b), ctypes.byref(h)), L)
        return Footer(BlockHandle(h[0], h[1]), BlockHandle(h[2], h[3]))


def seal_blocks(file, handles, types=None, stream=None):
    """Write type + masked crc trailers after every handle's extent, in place.
    file: uint8 CUDA tensor; handles: int64 CUDA tensor of shape (n, 2)."""
    L = _bind()
    n = handles.numel() // 2
    _check(L.lv_sst_seal_blocks_device(_dev_ptr(file, "file"), file.numel(), _dev_ptr(handles, "handles"),
                                       _dev_ptr(types, "types"), n, _stream_ptr(stream)))
    return file


def verify_blocks(file, handles, out_crc=False, stream=None):
    """Per-block status (BLOCK_OK / BLOCK_CHECKSUM_MISMATCH / BLOCK_OUT_OF_RANGE)
    as an int32 CUDA tensor; with out_crc also crc32c(contents||type)."""
    torch = _torch()
    L = _bind()
    n = handles.numel() // 2
    st = torch.empty(n, dtype=torch.int32, device=file.device)
    crc = torch.empty(n, dtype=torch.int32, device=file.device) if out_crc else None
    _check(L.lv_sst_verify_blocks_device(_dev_ptr(file, "file"), file.numel(), _dev_ptr(handles, "handles"), n,
                                         _dev_ptr(st, "status"), _dev_ptr(crc, "crc"), _stream_ptr(stream)))
    return (st, crc) if out_crc else st


def verify_blocks_host(file: bytes, handles, device: int = 0) -> np.ndarray:
    L = _bind()
    h = np.ascontiguousarray(handles, dtype=np.uint64).reshape(-1, 2)
    st = np.zeros(h.shape[0], dtype=np.uint32)
    buf = ctypes.create_string_buffer(bytes(file), max(len(file), 1))
    _check(L.lv_sst_verify_blocks_host(buf, len(file), h.ctypes.data, h.shape[0], st.ctypes.data, device))
    return st
