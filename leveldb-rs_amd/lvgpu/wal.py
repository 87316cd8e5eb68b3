"""Python mirror of the WAL record layer over the C ABI in include/lvgpu/wal.h.

    Scan.host(log, device)            GPU framing + CRC of every physical record
    scan_device(log_tensor, cap)      the same for a log already in HBM, no host sync
    Reader(log, scan, reporter, checksum, initial_offset)
                                      Reader::new / read_record / last_record_offset
                                      (log_reader.rs:75-120, :99)
    encode(records, dest_length)      Writer::add_record over many records with one
                                      GPU batch for the header CRCs (log_writer.rs:62-134)
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import LvError, lib

BLOCK_SIZE = 32768
HEADER_SIZE = 7
REC_OK, REC_BAD_LENGTH, REC_ZERO = 0, 1, 2

_REPORTER = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p)
_bound = False


def _bind():
    global _bound
    L = lib()
    if _bound:
        return L
    vp, sz, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64
    L.lv_wal_scan_host.restype = vp
    L.lv_wal_scan_host.argtypes = [vp, sz, ctypes.c_int]
    L.lv_wal_scan_host_pipelined.restype = vp
    L.lv_wal_scan_host_pipelined.argtypes = [vp, sz, ctypes.c_int]
    L.lv_wal_scan_wait.restype = ctypes.c_int
    L.lv_wal_scan_wait.argtypes = [vp]
    L.lv_wal_scan_count.restype = sz
    L.lv_wal_scan_count.argtypes = [vp]
    for f in ("lv_wal_scan_offsets", "lv_wal_scan_crcs", "lv_wal_scan_info"):
        getattr(L, f).restype = vp
        getattr(L, f).argtypes = [vp]
    L.lv_wal_scan_from_arrays.restype = vp
    L.lv_wal_scan_from_arrays.argtypes = [vp, vp, vp, sz]
    L.lv_wal_scan_free.restype = None
    L.lv_wal_scan_free.argtypes = [vp]
    L.lv_wal_reader_new.restype = vp
    L.lv_wal_reader_new.argtypes = [vp, sz, vp, _REPORTER, vp, ctypes.c_int, u64]
    L.lv_wal_reader_read_record.restype = ctypes.c_int
    L.lv_wal_reader_read_record.argtypes = [vp, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)]
    L.lv_wal_reader_last_record_offset.restype = u64
    L.lv_wal_reader_last_record_offset.argtypes = [vp]
    L.lv_wal_reader_free.restype = None
    L.lv_wal_reader_free.argtypes = [vp]
    L.lv_wal_scan_workspace_bytes.restype = sz
    L.lv_wal_scan_workspace_bytes.argtypes = [sz, sz]
    L.lv_wal_scan_device.restype = ctypes.c_int
    L.lv_wal_scan_device.argtypes = [vp, sz, vp, vp, vp, sz, vp, vp, sz, vp]
    L.lv_wal_encode_host.restype = ctypes.c_int
    L.lv_wal_encode_host.argtypes = [vp, vp, vp, sz, u64, vp, sz, ctypes.POINTER(ctypes.c_size_t), ctypes.c_int]
    _bound = True
    return L


def _err(what):
    raise LvError(f"{what}: {lib().lv_last_error().decode()}")


class Scan:
    """Physical records of a log with their CRC units' value()."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def host(cls, log: bytes, device: int = 0) -> "Scan":
        L = _bind()
        buf = ctypes.create_string_buffer(bytes(log), max(len(log), 1))
        h = L.lv_wal_scan_host(buf, len(log), device)
        if not h:
            _err("lv_wal_scan_host")
        return cls(h)

    @classmethod
    def host_pipelined(cls, log: bytes, device: int = 0) -> "Scan":
        """lv_wal_scan_host_pipelined: returns at once; a Reader over it waits
        only for the 32 MiB chunk holding its next header."""
        L = _bind()
        buf = ctypes.create_string_buffer(bytes(log), max(len(log), 1))
        h = L.lv_wal_scan_host_pipelined(buf, len(log), device)
        if not h:
            _err("lv_wal_scan_host_pipelined")
        s = cls(h)
        s._buf = buf  # the worker reads the log until the scan is freed
        return s

    def wait(self) -> None:
        if _bind().lv_wal_scan_wait(self._h):
            _err("lv_wal_scan_wait")

    @classmethod
    def from_arrays(cls, offsets, crcs, info) -> "Scan":
        L = _bind()
        o = np.ascontiguousarray(offsets, dtype=np.uint64)
        c = np.ascontiguousarray(crcs, dtype=np.uint32)
        i = np.ascontiguousarray(info, dtype=np.uint32)
        h = L.lv_wal_scan_from_arrays(o.ctypes.data, c.ctypes.data, i.ctypes.data, o.size)
        if not h:
            _err("lv_wal_scan_from_arrays")
        return cls(h)

    def _arr(self, fn, dtype):
        L = _bind()
        n = L.lv_wal_scan_count(self._h)
        if n == 0:
            return np.zeros(0, dtype=dtype)
        p = getattr(L, fn)(self._h)
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dtype))),
                                     shape=(n,)).copy()

    @property
    def offsets(self):
        return self._arr("lv_wal_scan_offsets", np.uint64)

    @property
    def crcs(self):
        return self._arr("lv_wal_scan_crcs", np.uint32)

    @property
    def info(self):
        return self._arr("lv_wal_scan_info", np.uint32)

    def __del__(self):
        if getattr(self, "_h", None):
            _bind().lv_wal_scan_free(self._h)
            self._h = None


def scan_device(log, cap: int, workspace=None, stream=None):
    """lv_wal_scan_device over a uint8 CUDA tensor holding the log (8-B
    aligned): returns (hdr_off int64, crc int32, info int32, count int64[1])
    CUDA tensors, asynchronous on `stream`.  count[0] > cap means the capacity
    was too small and nothing else was written."""
    import torch
    from . import LvError, _dev_ptr, _stream_ptr
    L = _bind()
    if log.dtype != torch.uint8:
        raise LvError(f"log must be a uint8 tensor (got {log.dtype}: numel() would not count bytes)")
    if workspace is not None and (workspace.dtype != torch.uint8 or workspace.device != log.device):
        raise LvError("workspace must be a uint8 tensor on the log's device")
    dev = log.device
    hdr = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
    crc = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
    info = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
    count = torch.empty(1, dtype=torch.int64, device=dev)
    need = L.lv_wal_scan_workspace_bytes(log.numel(), cap)
    if workspace is None:
        workspace = torch.empty(need, dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):  # the C call runs on the current device
        rc = L.lv_wal_scan_device(_dev_ptr(log, "log"), log.numel(), _dev_ptr(hdr, "hdr"), _dev_ptr(crc, "crc"),
                                  _dev_ptr(info, "info"), cap, _dev_ptr(count, "count"),
                                  _dev_ptr(workspace, "workspace"), workspace.numel(), _stream_ptr(stream))
    if rc != 0:
        _err("lv_wal_scan_device")
    return hdr, crc, info, count


def scan_workspace_bytes(nbytes: int, cap: int) -> int:
    return int(_bind().lv_wal_scan_workspace_bytes(nbytes, cap))


class Reader:
    """log_reader.rs Reader over an in-memory log whose CRCs come from `scan`.
    `reporter` needs .corruption(nbytes, reason) (log_reader.rs:37-42)."""

    def __init__(self, log: bytes, scan: Scan, reporter=None, checksum: bool = True, initial_offset: int = 0):
        L = _bind()
        self._log = ctypes.create_string_buffer(bytes(log), max(len(log), 1))
        self._scan = scan
        self._reporter = reporter

        def cb(_ctx, nbytes, reason):
            if self._reporter is not None:
                self._reporter.corruption(int(nbytes), reason.decode())
        self._cb = _REPORTER(cb)
        self._h = L.lv_wal_reader_new(self._log, len(log), scan._h if scan else None,
                                      self._cb if reporter is not None else _REPORTER(0), None,
                                      1 if checksum else 0, initial_offset)
        if not self._h:
            _err("lv_wal_reader_new")

    def read_record(self):
        """The next logical record (bytes), or None at end of input."""
        L = _bind()
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        rc = L.lv_wal_reader_read_record(self._h, ctypes.byref(p), ctypes.byref(n))
        if rc < 0:
            _err("lv_wal_reader_read_record")
        if rc == 0:
            return None
        return ctypes.string_at(p.value, n.value) if n.value else b""

    def last_record_offset(self) -> int:
        return int(_bind().lv_wal_reader_last_record_offset(self._h))

    def __del__(self):
        if getattr(self, "_h", None):
            _bind().lv_wal_reader_free(self._h)
            self._h = None


def encode(records, dest_length: int = 0, device: int = 0) -> bytes:
    """Bytes Writer::add_record appends for `records` (log_writer.rs:62-134),
    header CRCs computed in one GPU batch."""
    L = _bind()
    recs = [bytes(r) for r in records]
    payload = b"".join(recs)
    off = np.zeros(len(recs), dtype=np.uint64)
    ln = np.array([len(r) for r in recs], dtype=np.uint64)
    if len(recs) > 1:
        off[1:] = np.cumsum(ln[:-1])
    pbuf = ctypes.create_string_buffer(payload, max(len(payload), 1))
    need = ctypes.c_size_t()
    L.lv_wal_encode_host(pbuf, off.ctypes.data, ln.ctypes.data, len(recs), dest_length, None, 0,
                         ctypes.byref(need), device)
    out = ctypes.create_string_buffer(max(need.value, 1))
    rc = L.lv_wal_encode_host(pbuf, off.ctypes.data, ln.ctypes.data, len(recs), dest_length, out, need.value,
                              ctypes.byref(need), device)
    if rc != 0:
        _err("lv_wal_encode_host")
    return out.raw[: need.value]
