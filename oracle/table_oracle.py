"""ORACLE — TEST INFRASTRUCTURE ONLY.

Restatement of sunchao/leveldb-rs `src/table/format.rs` (BlockHandle, Footer)
and the varint coding it uses (`src/util/coding.rs:140-166, 206-251, 284-288`),
plus the SSTable block trailer the reference does not yet implement
(`options.rs:84` verify_checksums is declared but unused): upstream LevelDB's
`contents || type(1) || LE32(mask(crc32c(contents || type)))`, restated with
the reference crc32c (`crc32c_oracle.c`).

Pinning: BlockHandle/Footer by the reference's tests (`format.rs:107-147`)
and the varint tests (`coding.rs:481-510`), replayed in
tests/test_table_oracle.py.  The trailer layout has no reference code or
fixture: beyond the crc32c KATs it is **parity unpinned**.
Only tests/, smoke() and bench.py's cpu_baseline leg may import this module.
"""
from __future__ import annotations

import wal_oracle as W

TABLE_MAGIC_NUMBER = 0xDB4775248B80FB57           # format.rs:24
BLOCK_HANDLE_MAX_ENCODED_LENGTH = 10 + 10          # format.rs:35
FOOTER_ENCODED_LENGTH = 2 * BLOCK_HANDLE_MAX_ENCODED_LENGTH + 8  # format.rs:70
BLOCK_TRAILER_SIZE = 5                             # upstream table/format.h kBlockTrailerSize
NO_COMPRESSION = 0


class Corruption(Exception):
    pass


def varint_length(v: int) -> int:  # coding.rs:244-251
    n = 1
    while v >= 128:
        v >>= 7
        n += 1
    return n


def encode_varint_64(v: int) -> bytes:  # coding.rs:144-153
    out = bytearray()
    while v & 0xFFFFFFFFFFFFFF80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v & 0x7F)
    return bytes(out)


def decode_varint_64(src: bytes):  # coding.rs:223-241 (limit = len(src))
    shift = 0
    idx = 0
    result = 0
    while shift <= 63 and idx < len(src):
        byte = src[idx]
        idx += 1
        result |= ((byte & 0x7F) << shift) & 0xFFFFFFFFFFFFFFFF
        shift += 7
        if byte & 0x80 == 0:
            return result, idx
    raise Corruption("Error when decoding varint-64")


class BlockHandle:  # format.rs:26-50
    def __init__(self, offset: int, size: int):
        self.offset, self.size = offset, size

    def __eq__(self, o):
        return (self.offset, self.size) == (o.offset, o.size)

    def __repr__(self):
        return f"BlockHandle({self.offset}, {self.size})"

    def encode_to(self, dst: bytearray) -> None:  # :37-40
        dst += encode_varint_64(self.offset)
        dst += encode_varint_64(self.size)

    @staticmethod
    def decode_from(src: bytes):  # :42-49 -> (handle, bytes consumed)
        try:
            off, a = decode_varint_64(src)
            size, b = decode_varint_64(src[a:])
        except Corruption:
            raise Corruption("bad handle")
        return BlockHandle(off, size), a + b


class Footer:  # format.rs:52-104
    def __init__(self, metaindex_handle: BlockHandle, index_handle: BlockHandle):
        self.metaindex_handle, self.index_handle = metaindex_handle, index_handle

    def __eq__(self, o):
        return (self.metaindex_handle, self.index_handle) == (o.metaindex_handle, o.index_handle)

    def encode_to(self, dst: bytearray) -> None:  # :72-80
        original = len(dst)
        self.metaindex_handle.encode_to(dst)
        self.index_handle.encode_to(dst)
        # dst.resize(2 * MAX_ENCODED_LENGTH, 0): an absolute length, so the
        # assert below only holds for an empty dst (as in the reference)
        want = 2 * BLOCK_HANDLE_MAX_ENCODED_LENGTH
        if len(dst) < want:
            dst += bytes(want - len(dst))
        else:
            del dst[want:]
        dst += (TABLE_MAGIC_NUMBER & 0xFFFFFFFF).to_bytes(4, "little")
        dst += (TABLE_MAGIC_NUMBER >> 32).to_bytes(4, "little")
        assert len(dst) == original + FOOTER_ENCODED_LENGTH

    @staticmethod
    def decode_from(src: bytes) -> "Footer":  # :82-103
        magic_data = src[FOOTER_ENCODED_LENGTH - 8:]
        lo = W.decode_fixed_32(magic_data)
        hi = W.decode_fixed_32(magic_data[4:])
        if ((hi << 32) | lo) != TABLE_MAGIC_NUMBER:
            raise Corruption("not a sstable (bad magic number)")
        meta, a = BlockHandle.decode_from(src)
        index, _ = BlockHandle.decode_from(src[a:])
        return Footer(meta, index)


def block_trailer(contents: bytes, ctype: int = NO_COMPRESSION) -> bytes:
    """type || LE32(mask(crc32c(contents || type))) — parity unpinned (see header)."""
    crc = W.extend(W.value(contents), bytes([ctype]))
    return bytes([ctype]) + W.encode_fixed_32(W.mask(crc))


def verify_block(file: bytes, h: BlockHandle) -> int:
    """0 ok, 1 checksum mismatch, 2 handle out of range."""
    end = h.offset + h.size + BLOCK_TRAILER_SIZE
    if end > len(file):
        return 2
    stored = W.unmask(W.decode_fixed_32(file[h.offset + h.size + 1:end]))
    return 0 if stored == W.value(file[h.offset:h.offset + h.size + 1]) else 1
