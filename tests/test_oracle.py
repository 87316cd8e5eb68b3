"""Pins the CPU oracle (oracle/crc32c_oracle.c) to the reference's own tests:
crc32c.rs:147-171 (standard_results KATs) and :174-193 (values / extend /
mask properties), plus cross-checks sw == hw == bitwise on the golden cases."""
import ctypes
import os
import random
import subprocess

import pytest

from conftest import ROOT, kat_bytes
import wal_oracle as W


def test_oracle_builds():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    assert os.path.exists(os.path.join(ROOT, "oracle", "liblvoracle.so"))


def test_reference_kats(kat):
    ref = [k for k in kat["kats"] if k["source"].startswith("reference")]
    assert len(ref) == 5
    L = W.lib()
    for k in kat["kats"]:
        d = kat_bytes(k)
        assert W.value(d) == k["value"], k["name"]
        assert L.oracle_extend_sw(0, d, len(d)) == k["value"], k["name"]
        assert L.oracle_extend_hw(0, d, len(d)) == k["value"], k["name"]
        assert L.oracle_extend_bitwise(0, d, len(d)) == k["value"], k["name"]
        assert W.mask(k["value"]) == k["masked"]


def test_reference_properties(kat):
    p = kat["properties"]
    # crc32c.rs:174-176 values
    assert W.value(b"a") != W.value(b"foo")
    # crc32c.rs:179-184 extend
    assert W.value(b"hello world") == W.extend(W.value(b"hello "), b"world")
    # crc32c.rs:187-193 mask
    crc = W.value(b"foo")
    assert W.mask(crc) != crc
    assert W.mask(W.mask(crc)) != crc
    assert W.unmask(W.mask(crc)) == crc
    assert W.unmask(W.unmask(W.mask(W.mask(crc)))) == crc
    assert p["mask_of_foo"] == W.mask(crc)
    assert p["type_crc"] == [0x527d5351, 0xa016d052, 0xb34623a6, 0x412da0a5, 0x95e7c44e]
    assert W.extend(0x12345678, b"") == 0x12345678


def test_golden_cases(kat, arena):
    L = W.lib()
    for off, ln, seed, crc, masked in kat["cases"]:
        d = arena[off:off + ln]
        assert L.oracle_extend_hw(seed, d, ln) == crc
        assert L.oracle_extend_sw(seed, d, ln) == crc
        assert W.mask(crc) == masked


def test_unaligned_and_batch(arena):
    """extend_hw's alignment prologue (crc32c.rs:97-102) must not change results;
    oracle_batch must equal per-buffer calls."""
    import numpy as np
    L = W.lib()
    rng = random.Random(7)
    buf = ctypes.create_string_buffer(arena[:70000], 70000)
    base = ctypes.addressof(buf)
    offs, lens, seeds = [], [], []
    for _ in range(400):
        o = rng.randrange(0, 65000)
        n = rng.randrange(0, 4000)
        n = min(n, 70000 - o)
        s = rng.getrandbits(32)
        p = ctypes.cast(base + o, ctypes.c_char_p)
        a = L.oracle_extend_hw(s, p, n)
        b = L.oracle_extend_sw(s, p, n)
        c = L.oracle_extend_bitwise(s, p, n)
        assert a == b == c
        offs.append(o), lens.append(n), seeds.append(s)
    o = np.array(offs, dtype=np.uint64)
    ln = np.array(lens, dtype=np.uint32)
    sd = np.array(seeds, dtype=np.uint32)
    out = np.zeros(len(offs), dtype=np.uint32)
    L.oracle_batch(base, o.ctypes.data, ln.ctypes.data, sd.ctypes.data, out.ctypes.data, len(offs), 1)
    for i in range(len(offs)):
        p = ctypes.cast(base + offs[i], ctypes.c_char_p)
        assert out[i] == W.mask(L.oracle_extend(seeds[i], p, lens[i]))


def test_table16_matches_make_table():
    """TABLE16 row 0 is make_table(CASTAGNOLI_POLY) (crc32c.rs:27-28,126-140)."""
    import numpy as np
    t = np.zeros(16 * 256, dtype=np.uint32)
    W.lib().oracle_table16(t.ctypes.data)
    t = t.reshape(16, 256)
    assert t[0][1] == 0xf26b8303  # first nontrivial entry of the Castagnoli table
    for j in range(1, 16):
        for i in (0, 1, 127, 255):
            c = int(t[j - 1][i])
            assert t[j][i] == (c >> 8) ^ int(t[0][c & 0xFF])


def test_random_module():
    """random.rs:80-88 KAT (drives the WAL size distribution)."""
    r = W.Random(0)
    assert r.seed == 1
    r = W.Random(2147483647)
    assert r.seed == 1
    r = W.Random(3)
    assert r.next() == 50421
    assert r.uniform(10) == 7
    assert r.skewed(2) == 1


@pytest.mark.parametrize("n", [0, 1, 3, 4, 7, 8, 15, 16, 17, 31, 33, 4096])
def test_splitmix_fill_is_prefix_consistent(n):
    L = W.lib()
    full = ctypes.create_string_buffer(64 + n)
    L.oracle_fill_splitmix(full, 0, 64 + n, 99)
    part = ctypes.create_string_buffer(n)
    L.oracle_fill_splitmix(part, 13, n, 99)
    assert part.raw[:n] == full.raw[13:13 + n]


def _reader_counts(log: bytes):
    """(passed, mismatched, bad length) physical records per the Python
    restatement of log_reader.rs:271-364: scan_log walks every header; the
    reference drops the rest of a block after a mismatch and counts an
    overrun as "bad record length" only before EOF."""
    offs, crcs, info = W.scan_log(log)
    ok = mm = bl = 0
    dropped = set()
    last_block = (len(log) - 1) // W.BLOCK_SIZE if log else -1
    short_tail = len(log) % W.BLOCK_SIZE != 0
    for o, c, i in zip(offs, crcs, info):
        blk = o // W.BLOCK_SIZE
        if blk in dropped:
            continue
        status = (i >> 8) & 0xFF
        if status == 1:
            if not (blk == last_block and short_tail):
                bl += 1
            continue
        if status == 2:
            continue
        if W.unmask(W.decode_fixed_32(log[o:o + 4])) == c:
            ok += 1
        else:
            mm += 1
            dropped.add(blk)
    return ok, mm, bl


def test_wal_verify_oracle_matches_reader_restatement():
    """oracle_wal_verify (verify_oracle.c, the bench's WAL cpu_baseline) counts
    what the Python reader restatement counts, on intact, corrupted and
    truncated logs written by the oracle Writer."""
    L = W.lib()
    rnd = W.Random(301)
    rng = random.Random(17)
    seen_bl = seen_mm = False
    for trial in range(12):
        dest = bytearray()
        w = W.Writer(dest)
        for i in range(60):
            w.add_record(W.random_skewed_string(i, rnd).encode())
        log = bytearray(dest)
        for _ in range(trial % 4):  # corrupt payload / header bytes
            k = rng.randrange(len(log))
            log[k] ^= 1 << rng.randrange(8)
        if trial % 3 == 2:
            log = log[:rng.randrange(len(log))]
        if trial % 4 == 1 and len(log) > 3 * W.BLOCK_SIZE:  # a length that overruns block 1
            log[W.BLOCK_SIZE + 5] = 0x7F
        buf = (ctypes.c_uint8 * max(len(log), 1)).from_buffer_copy(bytes(log) or b"\0")
        mm, bl = ctypes.c_uint64(), ctypes.c_uint64()
        ok = L.oracle_wal_verify(ctypes.addressof(buf), len(log), ctypes.byref(mm), ctypes.byref(bl))
        assert (ok, mm.value, bl.value) == _reader_counts(bytes(log)), trial
        seen_bl = seen_bl or bl.value > 0
        seen_mm = seen_mm or mm.value > 0
    assert seen_bl and seen_mm


def test_units_seal_and_verify_oracle():
    """oracle_units_seal writes type || LE32(mask(crc32c(contents || type)))
    and oracle_units_verify finds exactly the trailers that were damaged."""
    import numpy as np
    L = W.lib()
    rng = np.random.default_rng(3)
    sizes = rng.integers(0, 5000, 200).astype(np.uint32)
    offs = np.zeros(200, dtype=np.uint64)
    offs[1:] = np.cumsum(sizes[:-1].astype(np.uint64) + 5)
    f = rng.integers(0, 256, int(offs[-1] + sizes[-1] + 5), dtype=np.uint8)
    L.oracle_units_seal(f.ctypes.data, offs.ctypes.data, sizes.ctypes.data, 200)
    for i in (0, 57, 199):
        o, s = int(offs[i]), int(sizes[i])
        assert W.decode_fixed_32(f[o + s + 1:o + s + 5].tobytes()) == W.mask(W.value(f[o:o + s + 1].tobytes()))
    uo, ul, co = offs.copy(), sizes + 1, offs + sizes + 1
    assert L.oracle_units_verify(f.ctypes.data, uo.ctypes.data, ul.ctypes.data, co.ctypes.data, 200) == 0
    f[int(co[9])] ^= 4
    f[int(uo[100])] ^= 1 if sizes[100] else 0
    bad = 1 + (1 if sizes[100] else 0)
    assert L.oracle_units_verify(f.ctypes.data, uo.ctypes.data, ul.ctypes.data, co.ctypes.data, 200) == bad
