"""ORACLE — TEST INFRASTRUCTURE ONLY.

Pure-Python restatement of the reference write-ahead-log record layer of
sunchao/leveldb-rs (`src/log_writer.rs`, `src/log_reader.rs`,
`src/log_format.rs`) and its deterministic RNG (`src/util/random.rs`), used
to (a) generate the WAL golden fixtures under `tests/golden/` and (b) check
the GPU batched WAL encode / verify paths.  CRCs come from the C oracle
(`crc32c_oracle.c`).  Only tests, `__graft_entry__.smoke()` and `bench.py`'s
cpu_baseline leg may import this module.

Pinned by the reference's own WAL tests (`log_writer.rs:445-838`), replayed in
`tests/test_wal_log.py` (and `tests/test_wal_boundary.py` for the host reader).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))

# log_format.rs:22-29, 62-66
ZERO, FULL, FIRST, MIDDLE, LAST = 0, 1, 2, 3, 4
MAX_RECORD_TYPE = LAST
BLOCK_SIZE = 32768
HEADER_SIZE = 7
# log_reader.rs:27-34
EOF = MAX_RECORD_TYPE + 1
BAD_RECORD = MAX_RECORD_TYPE + 2

_lib = None


def lib():
    """Load the C oracle (built by `make -C oracle`)."""
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, "liblvoracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle not built: run `make -C oracle`")
        L = ctypes.CDLL(path)
        u32, sz, p = ctypes.c_uint32, ctypes.c_size_t, ctypes.c_void_p
        for name in ("oracle_value",):
            getattr(L, name).restype = u32
            getattr(L, name).argtypes = [ctypes.c_char_p, sz]
        for name in ("oracle_extend", "oracle_extend_sw", "oracle_extend_hw", "oracle_extend_bitwise"):
            getattr(L, name).restype = u32
            getattr(L, name).argtypes = [u32, ctypes.c_char_p, sz]
        for name in ("oracle_mask", "oracle_unmask"):
            getattr(L, name).restype = u32
            getattr(L, name).argtypes = [u32]
        for name in ("oracle_batch", "oracle_batch_sw"):
            getattr(L, name).restype = None
            getattr(L, name).argtypes = [p, p, p, p, p, sz, u32]
        L.oracle_bench_loop.restype = u32
        L.oracle_bench_loop.argtypes = [p, sz, ctypes.c_uint64, ctypes.c_int]
        L.oracle_fill_splitmix.restype = None
        L.oracle_fill_splitmix.argtypes = [p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_table16.restype = None
        L.oracle_table16.argtypes = [p]
        L.oracle_wal_verify.restype = ctypes.c_uint64  # verify_oracle.c
        L.oracle_wal_verify.argtypes = [p, ctypes.c_uint64, p, p]
        L.oracle_units_verify.restype = ctypes.c_uint64
        L.oracle_units_verify.argtypes = [p, p, p, p, sz]
        L.oracle_units_seal.restype = None
        L.oracle_units_seal.argtypes = [p, p, p, sz]
        L.oracle_hash_batch.restype = None  # hash_oracle.c
        L.oracle_hash_batch.argtypes = [p] * 5 + [sz]
        _lib = L
    return _lib


def value(b: bytes) -> int:  # crc32c.rs:40
    return lib().oracle_value(bytes(b), len(b))


def extend(c: int, b: bytes) -> int:  # crc32c.rs:42-51
    return lib().oracle_extend(c, bytes(b), len(b))


def mask(c: int) -> int:  # crc32c.rs:53-57
    return lib().oracle_mask(c)


def unmask(c: int) -> int:  # crc32c.rs:59-63
    return lib().oracle_unmask(c)


def encode_fixed_32(v: int) -> bytes:  # coding.rs:32-38
    return int(v & 0xFFFFFFFF).to_bytes(4, "little")


def decode_fixed_32(b: bytes) -> int:  # coding.rs:70-77
    return int.from_bytes(bytes(b[:4]), "little")


class Random:
    """random.rs:19-70 — Park–Miller MCG (a = 16807, m = 2^31 - 1)."""

    def __init__(self, s: int):
        seed = s & 0x7FFFFFFF
        if seed == 0 or seed == 2147483647:
            seed = 1
        self.seed = seed

    def next(self) -> int:  # random.rs:38-51
        m = 2147483647
        product = self.seed * 16807
        s = ((product >> 31) + (product & m)) & 0xFFFFFFFF
        if s > m:
            s -= m
        self.seed = s
        return s

    def uniform(self, n: int) -> int:  # random.rs:55
        return self.next() % n

    def one_in(self, n: int) -> bool:  # random.rs:59
        return self.next() % n == 0

    def skewed(self, max_log: int) -> int:  # random.rs:66-69
        r = 1 << self.uniform(max_log + 1)
        return self.uniform(r)


class Writer:
    """log_writer.rs:28-143."""

    def __init__(self, dest: bytearray, dest_length: int = 0):
        self.dest = dest
        self.block_offset = dest_length % BLOCK_SIZE  # log_writer.rs:48-56
        # init_type_crc, log_writer.rs:136-142
        self.type_crc = [value(bytes([t])) for t in range(MAX_RECORD_TYPE + 1)]

    def add_record(self, data: bytes) -> None:  # log_writer.rs:62-110
        data = bytes(data)
        left = len(data)
        pos = 0
        begin = True
        while True:
            leftover = BLOCK_SIZE - self.block_offset
            if leftover < HEADER_SIZE:
                if leftover > 0:
                    self.dest += b"\x00" * leftover
                self.block_offset = 0
            avail = BLOCK_SIZE - self.block_offset - HEADER_SIZE
            frag = left if left < avail else avail
            end = left == frag
            if begin and end:
                t = FULL
            elif begin:
                t = FIRST
            elif end:
                t = LAST
            else:
                t = MIDDLE
            self.emit_physical_record(t, data[pos:pos + frag])
            pos += frag
            left -= frag
            begin = False
            if left <= 0:
                break

    def emit_physical_record(self, t: int, data: bytes) -> None:  # log_writer.rs:112-134
        n = len(data)
        assert n <= 0xFFFF
        assert self.block_offset + HEADER_SIZE + n <= BLOCK_SIZE
        crc = mask(extend(self.type_crc[t], data))
        self.dest += encode_fixed_32(crc) + bytes([n & 0xFF, n >> 8, t]) + data
        self.block_offset += HEADER_SIZE + n


class StringSource:
    """log_writer.rs:180-223 (test in-memory SequentialFile)."""

    def __init__(self, contents: bytes = b""):
        self.contents = bytes(contents)
        self.pos = 0
        self.force_error = False
        self.returned_partial = False

    def read(self, n: int):
        assert not self.returned_partial, "must not read() after eof/error"
        if self.force_error:
            self.force_error = False
            self.returned_partial = True
            return None  # error
        avail = len(self.contents) - self.pos
        if avail < n:
            n = avail
            self.returned_partial = True
        r = self.contents[self.pos:self.pos + n]
        self.pos += n
        return r

    def skip(self, n: int) -> bool:
        if n > len(self.contents) - self.pos:
            self.pos = len(self.contents)
            return False
        self.pos += n
        return True


class ReportCollector:
    """log_writer.rs:225-244."""

    def __init__(self):
        self.dropped_bytes = 0
        self.message = ""

    def corruption(self, nbytes: int, reason: str) -> None:
        self.dropped_bytes += nbytes
        self.message += reason


class Reader:
    """log_reader.rs:44-393.  `buffer` is kept as (bytes, start) like the
    reference's Slice view over `backing_store`."""

    def __init__(self, source: StringSource, reporter, checksum: bool, initial_offset: int):
        self.file = source
        self.reporter = reporter
        self.checksum = checksum
        self.buf = b""
        self.eof = False
        self.last_record_offset = 0
        self.end_of_buffer_offset = 0
        self.initial_offset = initial_offset
        self.resyncing = initial_offset > 0
        # CRC calls made by read_physical_record: list of (crc_bytes, expected)
        self.crc_calls = []

    def _report_drop(self, nbytes: int, reason: str) -> None:  # log_reader.rs:101-109
        if self.reporter is not None:
            if self.end_of_buffer_offset >= len(self.buf) + nbytes + self.initial_offset:
                self.reporter.corruption(nbytes, reason)

    def read_record(self):  # log_reader.rs:120-265
        if self.last_record_offset < self.initial_offset:
            if not self._skip_to_initial_block():
                return None
        scratch = bytearray()
        in_frag = False
        prospective = 0
        while True:
            rtype, frag = self._read_physical_record()
            fsize = len(frag) if frag is not None else 0
            phys = self.end_of_buffer_offset - len(self.buf) - HEADER_SIZE - fsize
            if self.resyncing:
                if rtype == MIDDLE:
                    continue
                elif rtype == LAST:
                    self.resyncing = False
                    continue
                else:
                    self.resyncing = False
            if rtype == EOF:
                if in_frag:
                    scratch.clear()
                return None
            elif rtype == BAD_RECORD:
                if in_frag:
                    self._report_drop(len(scratch), "error in middle of record")
                    in_frag = False
                    scratch.clear()
            else:
                scratch_size = len(scratch) if in_frag else 0
                if rtype == FULL:
                    if in_frag:
                        self._report_drop(len(scratch), "partial record without end(1)")
                    prospective = phys
                    self.last_record_offset = prospective
                    return bytes(frag)
                elif rtype == FIRST:
                    if in_frag:
                        self._report_drop(len(scratch), "partial record without end(2)")
                    prospective = phys
                    scratch = bytearray(frag)
                    in_frag = True
                elif rtype == MIDDLE:
                    if not in_frag:
                        self._report_drop(len(frag), "missing start of fragmented record(1)")
                    else:
                        scratch += frag
                elif rtype == LAST:
                    if not in_frag:
                        self._report_drop(len(frag), "missing start of fragmented record(2)")
                    else:
                        scratch += frag
                        self.last_record_offset = prospective
                        return bytes(scratch)
                elif rtype == ZERO:
                    self._report_drop(len(frag) + scratch_size, "unexpected record type")
                    in_frag = False
                    scratch.clear()
                else:
                    self._report_drop(len(frag) + scratch_size, "unknown record type")
                    in_frag = False
                    scratch.clear()

    def _read_physical_record(self):  # log_reader.rs:271-364
        while True:
            if len(self.buf) < HEADER_SIZE:
                if not self.eof:
                    self.buf = b""
                    r = self.file.read(BLOCK_SIZE)
                    if r is None:
                        self._report_drop(BLOCK_SIZE, "read error")
                        self.eof = True
                        return EOF, None
                    self.end_of_buffer_offset += len(r)
                    self.buf = r
                    if len(self.buf) < BLOCK_SIZE:
                        self.eof = True
                    continue
                else:
                    self.buf = b""
                    return EOF, None
            header = self.buf
            length = header[4] | (header[5] << 8)
            t = header[6]
            if HEADER_SIZE + length > len(self.buf):
                drop = len(self.buf)
                self.buf = b""
                if not self.eof:
                    self._report_drop(drop, "bad record length")
                    return BAD_RECORD, None
                return EOF, None
            if t == ZERO and length == 0:
                self.buf = b""
                return BAD_RECORD, None
            if self.checksum:
                expected = unmask(decode_fixed_32(header))
                actual = value(header[6:7 + length])
                self.crc_calls.append((bytes(header[6:7 + length]), expected))
                if expected != actual:
                    drop = len(self.buf)
                    self.buf = b""
                    self._report_drop(drop, "checksum mismatch")
                    return BAD_RECORD, None
            frag = header[HEADER_SIZE:HEADER_SIZE + length]
            self.buf = self.buf[HEADER_SIZE + length:]
            if self.end_of_buffer_offset - len(self.buf) - HEADER_SIZE - length < self.initial_offset:
                return BAD_RECORD, None
            return t, frag

    def _skip_to_initial_block(self) -> bool:  # log_reader.rs:369-392
        off_in_block = self.initial_offset % BLOCK_SIZE
        start = self.initial_offset - off_in_block
        if off_in_block > BLOCK_SIZE - 6:
            start += BLOCK_SIZE
        self.end_of_buffer_offset = start
        if start > 0:
            if not self.file.skip(start):
                self._report_drop(start, "skip error")
                return False
        return True


def big_string(partial: str, n: int) -> str:  # log_writer.rs:447-454
    out = ""
    while len(out) < n:
        out += partial
    return out[:n]


def random_skewed_string(i: int, rnd: Random) -> str:  # log_writer.rs:456-458
    return big_string(str(i), rnd.skewed(17))


def wal_physical_records(log: bytes):
    """Parse a well-formed log into its physical records without verifying:
    returns a list of (header_offset, length, type).  Mirrors the framing of
    log_reader.rs:271-331 (trailer skip < HEADER_SIZE, ZERO/len-0 skip)."""
    out = []
    pos = 0
    n = len(log)
    while pos < n:
        block_left = BLOCK_SIZE - (pos % BLOCK_SIZE)
        if block_left < HEADER_SIZE:
            pos += block_left
            continue
        if pos + HEADER_SIZE > n:
            break
        length = log[pos + 4] | (log[pos + 5] << 8)
        t = log[pos + 6]
        if pos + HEADER_SIZE + length > n or HEADER_SIZE + length > block_left:
            break
        if not (t == ZERO and length == 0):
            out.append((pos, length, t))
        pos += HEADER_SIZE + length
    return out


def scan_log(log: bytes):
    """Restatement of the block framing of log_reader.rs:271-331 over a whole
    log, as the GPU scan computes it: per 32 KiB block, walk the header chain
    until < HEADER_SIZE bytes remain, a length overruns the block (status 1)
    or a ZERO/0 header (status 2).  Returns (header offsets, value([type ||
    payload]) or 0, info = type | status << 8 | length << 16)."""
    offs, crcs, info = [], [], []
    for start in range(0, len(log), BLOCK_SIZE):
        blen = min(BLOCK_SIZE, len(log) - start)
        pos = 0
        while blen - pos >= HEADER_SIZE:
            h = log[start + pos:start + pos + HEADER_SIZE]
            length = h[4] | (h[5] << 8)
            t = h[6]
            status = 0
            if HEADER_SIZE + length > blen - pos:
                status = 1
            elif t == ZERO and length == 0:
                status = 2
            offs.append(start + pos)
            crcs.append(value(log[start + pos + 6:start + pos + 7 + length]) if status == 0 else 0)
            info.append(t | (status << 8) | (length << 16))
            if status:
                break
            pos += HEADER_SIZE + length
    return offs, crcs, info
