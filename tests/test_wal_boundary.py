"""CPU checks of the WAL C ABI (include/lvgpu/wal.h) that need no GPU: scan
containers built from arrays, the host Reader's refusal of a header its scan
does not cover, and the oracle's block framing (scan_log) against the
reference fixture."""
import numpy as np
import pytest

import wal_oracle as W


def _log(msgs):
    d = bytearray()
    w = W.Writer(d)
    for m in msgs:
        w.add_record(m)
    return bytes(d)


def test_scan_from_arrays_roundtrip():
    import lvgpu.wal as LW
    o, c, i = W.scan_log(_log([b"foo", b"x" * 70000, b""]))
    s = LW.Scan.from_arrays(o, c, i)
    assert s.offsets.tolist() == o and s.crcs.tolist() == c and s.info.tolist() == i
    e = LW.Scan.from_arrays([], [], [])
    assert e.offsets.size == 0


def test_scan_log_matches_fixture_framing(wal_golden):
    for sc in wal_golden["scenarios"]:
        if sc["log_hex"] is None or sc["physical_records"] is None or sc["dropped_bytes"]:
            continue
        log = bytes.fromhex(sc["log_hex"])
        o, c, i = W.scan_log(log)
        ok = [(o[k], i[k] >> 16, i[k] & 0xFF) for k in range(len(o)) if (i[k] >> 8) & 0xFF == W_OK]
        assert [list(r) for r in ok] == sc["physical_records"]
        for k in range(len(o)):  # stored masked CRC == mask(value(unit)) for an intact log
            if (i[k] >> 8) & 0xFF == W_OK:
                assert W.mask(c[k]) == W.decode_fixed_32(log[o[k]:o[k] + 4])


W_OK = 0


def test_reader_rejects_uncovered_header():
    import lvgpu
    import lvgpu.wal as LW
    log = _log([b"foo", b"bar"])
    o, c, i = W.scan_log(log)
    r = LW.Reader(log, LW.Scan.from_arrays(o[:1], c[:1], i[:1]), W.ReportCollector())
    assert r.read_record() == b"foo"
    with pytest.raises(lvgpu.LvError):
        r.read_record()


def test_reader_checksum_off_ignores_crcs():
    import lvgpu.wal as LW
    log = _log([b"foo", b"bar"])
    o, c, i = W.scan_log(log)
    rep = W.ReportCollector()
    r = LW.Reader(log, LW.Scan.from_arrays(o, [x ^ 1 for x in c], i), rep, checksum=False)
    assert [r.read_record(), r.read_record(), r.read_record()] == [b"foo", b"bar", None]
    rep2 = W.ReportCollector()
    r2 = LW.Reader(log, LW.Scan.from_arrays(o, [x ^ 1 for x in c], i), rep2, checksum=True)
    assert r2.read_record() is None and "checksum mismatch" in rep2.message


def test_native_reader_replay_helper():
    """tools/host_replay.c (bench.py --wal's native Reader loop) reads every
    logical record of a log through the C ABI, from a scan built from the
    oracle's CRCs (no GPU needed)."""
    import ctypes
    import os
    import lvgpu.wal as LW
    from conftest import ROOT
    rnd = W.Random(301)
    msgs = [W.random_skewed_string(i, rnd).encode() for i in range(200)]
    log = _log(msgs)
    o, c, i = W.scan_log(log)
    s = LW.Scan.from_arrays(o, c, i)
    R = ctypes.CDLL(os.path.join(ROOT, "leveldb-rs_amd", "lib", "libhostreplay.so"))
    R.lv_replay_reader.restype = ctypes.c_double
    R.lv_replay_reader.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    nr, nb = ctypes.c_uint64(), ctypes.c_uint64()
    t = R.lv_replay_reader(log, len(log), s._h, 2, ctypes.byref(nr), ctypes.byref(nb))
    assert t >= 0 and nr.value == len(msgs) and nb.value == sum(len(m) for m in msgs)
