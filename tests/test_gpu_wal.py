"""GPU WAL paths against the oracle.

  lv_wal_scan_host   == oracle.scan_log (framing + value() of every unit),
                        on intact, corrupted, truncated, zero-padded and
                        random-garbage logs;
  lv_wal_encode_host == oracle Writer bytes for many records at once, at
                        every interesting dest_length (block-trailer edges).
The full reference WAL suite over these two paths is tests/test_wal_log.py
(backend "gpu")."""
import numpy as np
import pytest

import wal_oracle as W

pytestmark = pytest.mark.gpu
B, H = W.BLOCK_SIZE, W.HEADER_SIZE


def _oracle_encode(recs, dest_length=0):
    d = bytearray()
    w = W.Writer(d, dest_length)
    for r in recs:
        w.add_record(r)
    return bytes(d)


def _random_records(rng, n, maxlog=17):
    out = []
    for _ in range(n):
        ln = int(rng.integers(0, 1 << int(rng.integers(0, maxlog + 1))))
        out.append(rng.integers(0, 256, size=ln, dtype=np.uint8).tobytes())
    return out


def _check_scan(log):
    import lvgpu.wal as LW
    o, c, i = W.scan_log(log)
    for s in (LW.Scan.host(log), LW.Scan.host_pipelined(log)):
        assert s.offsets.tolist() == o
        assert s.info.tolist() == i
        assert s.crcs.tolist() == c


def test_scan_small_logs(gpu):
    _check_scan(b"")
    for n in range(1, 40):
        _check_scan(_oracle_encode([b"ab" * n])[: n + 3])
    _check_scan(_oracle_encode([b"foo", b"", b"bar" * 11000, b"x"]))


def test_scan_random_logs(gpu):
    rng = np.random.default_rng(17)
    for trial in range(6):
        log = bytearray(_oracle_encode(_random_records(rng, 300), int(rng.integers(0, 2 * B))))
        if trial >= 2:  # corruption: flipped bytes, including headers
            for pos in rng.integers(0, len(log), size=20):
                log[int(pos)] ^= int(rng.integers(1, 256))
        if trial >= 4:
            del log[len(log) - int(rng.integers(1, 5000)):]
        _check_scan(bytes(log))


def test_scan_zero_padding_and_garbage(gpu):
    rng = np.random.default_rng(3)
    log = _oracle_encode(_random_records(rng, 50)) + bytes(3 * B + 123)  # preallocated tail
    _check_scan(log)
    _check_scan(rng.integers(0, 256, size=5 * B + 77, dtype=np.uint8).tobytes())
    _check_scan(bytes(B * 2))


def test_scan_large_log(gpu):
    """A 64 MiB log of ~46k skewed records: scan equals the oracle's."""
    rng = np.random.default_rng(11)
    recs = _random_records(rng, 12000, maxlog=14)
    log = _oracle_encode(recs)
    _check_scan(log)


@pytest.mark.parametrize("dest_length", [0, 1, B - H - 1, B - H, B - H + 1, B - 1, B, 5 * B + 17])
def test_encode_matches_writer(gpu, dest_length):
    import lvgpu.wal as LW
    rng = np.random.default_rng(dest_length)
    recs = [b"", b"foo"] + _random_records(rng, 200) + [bytes(3 * B + 5), b""]
    got = LW.encode(recs, dest_length=dest_length)
    assert got == _oracle_encode(recs, dest_length)


def test_encode_empty_batch(gpu):
    import lvgpu.wal as LW
    assert LW.encode([]) == b""
    # records with no payload bytes at all: every fragment CRC covers zero bytes
    empties = [b""] * 5
    for dest_length in (0, B - H - 2):
        assert LW.encode(empties, dest_length=dest_length) == _oracle_encode(empties, dest_length)


def test_pipelined_scan_reader_over_chunks(gpu):
    """lv_wal_scan_host_pipelined over a log of several 32 MiB chunks: the
    Reader replays every record while later chunks are still being scanned
    (it waits per chunk), with no reports; the finished scan's arrays equal
    lv_wal_scan_host's.  Corrupted bytes in the second chunk are reported the
    same way by both scans' readers."""
    import lvgpu.wal as LW
    rng = np.random.default_rng(41)
    recs = _random_records(rng, 24000, maxlog=16)
    log = LW.encode(recs)
    assert len(log) > 2 * (32 << 20)
    rep = W.ReportCollector()
    r = LW.Reader(log, LW.Scan.host_pipelined(log), rep)
    for want in recs:
        assert r.read_record() == want
    assert r.read_record() is None
    assert rep.dropped_bytes == 0 and rep.message == ""
    a, b = LW.Scan.host(log), LW.Scan.host_pipelined(log)
    b.wait()
    assert np.array_equal(a.offsets, b.offsets) and np.array_equal(a.crcs, b.crcs)
    assert np.array_equal(a.info, b.info)
    bad = bytearray(log)
    for pos in rng.integers(33 << 20, 40 << 20, size=10):
        bad[int(pos)] ^= 0x5A
    bad = bytes(bad)
    got = []
    for scan in (LW.Scan.host(bad), LW.Scan.host_pipelined(bad)):
        rep = W.ReportCollector()
        rd = LW.Reader(bad, scan, rep)
        n = 0
        while rd.read_record() is not None:
            n += 1
        got.append((n, rep.dropped_bytes, rep.message))
    assert got[0] == got[1] and got[0][1] > 0


def test_pipelined_scan_worker_error_surfaces(gpu):
    """a pipelined scan whose worker fails (here: a device ordinal
    past the last GPU) reports the worker's error from lv_wal_scan_wait and
    from the accessors (count 0), and a Reader over it fails with that error
    instead of returning end of input."""
    import torch

    import lvgpu
    import lvgpu.wal as LW
    log = LW.encode([bytes([i % 251]) * (100 + i) for i in range(50)])
    bad_dev = torch.cuda.device_count() + 3
    s = LW.Scan.host_pipelined(log, device=bad_dev)
    with pytest.raises(lvgpu.LvError) as e:
        s.wait()
    assert "WAL scan" in str(e.value)
    assert LW._bind().lv_wal_scan_count(s._h) == 0
    s2 = LW.Scan.host_pipelined(log, device=bad_dev)
    rd = LW.Reader(log, s2, W.ReportCollector())
    with pytest.raises(lvgpu.LvError) as e2:
        rd.read_record()
    assert "WAL scan" in str(e2.value)
    # the library still works on a valid device afterwards
    r = LW.Reader(log, LW.Scan.host_pipelined(log))
    assert r.read_record() == bytes([0]) * 100


def test_encode_then_scan_then_read(gpu):
    """Round trip at scale: GPU encode -> GPU scan -> host reader returns the
    records, with no reports."""
    import lvgpu.wal as LW
    rng = np.random.default_rng(23)
    recs = _random_records(rng, 3000, maxlog=16)
    log = LW.encode(recs)
    rep = W.ReportCollector()
    r = LW.Reader(log, LW.Scan.host(log), rep)
    for want in recs:
        assert r.read_record() == want
    assert r.read_record() is None
    assert rep.dropped_bytes == 0 and rep.message == ""


SORTED = "wal_hist+sort_scan+wal_scatter+crc32c_classes_kernel"


def _check_scan_device(log, cap=None, shift=0):
    """shift: the log's offset from a 16-B boundary (the scan needs 8-B
    alignment)."""
    import lvgpu
    import lvgpu.wal as LW
    import torch
    o, c, i = W.scan_log(log)
    cap = len(o) if cap is None else cap
    t = torch.frombuffer(bytes(shift) + bytes(log) + b"\0", dtype=torch.uint8).to("cuda:0")[shift:shift + len(log)]
    assert len(log) == 0 or t.data_ptr() % 16 == shift
    # twice: a fresh workspace, then one left dirty (0xff): the scan reads
    # nothing of the workspace it did not write first
    dirty = torch.full((LW.scan_workspace_bytes(len(log), cap),), 0xff, dtype=torch.uint8, device="cuda:0")
    kern = SORTED + ("+wal_unsort" if cap else "")
    for ws in (None, dirty):
        hdr, crc, info, count = LW.scan_device(t, cap, workspace=ws)
        torch.cuda.synchronize()
        assert lvgpu.last_kernel() == kern or len(log) == 0, lvgpu.last_kernel()
        n = int(count.item())
        assert n == len(o), (n, len(o))
        if n <= cap:
            assert hdr[:n].cpu().numpy().tolist() == o
            assert info[:n].cpu().numpy().view(np.uint32).tolist() == i
            assert crc[:n].cpu().numpy().view(np.uint32).tolist() == c


@pytest.mark.parametrize("shift", [0, 8])
def test_scan_device_matches_oracle(gpu, shift):
    """lv_wal_scan_device (log already in HBM, framing fused into the length
    sort, no host sync) == oracle.scan_log on intact, corrupted, truncated,
    zero-padded, garbage and odd-length logs, 16-B and 8-B aligned."""
    rng = np.random.default_rng(29)
    _check_scan_device(b"", shift=shift)
    for n in (1, 5, 6, 7, 8, 13):
        _check_scan_device(_oracle_encode([b"ab" * n])[: n + 3], shift=shift)
    _check_scan_device(_oracle_encode([b"foo", b"", b"bar" * 11000, b"x"]), shift=shift)
    for trial in range(4):
        log = bytearray(_oracle_encode(_random_records(rng, 400), int(rng.integers(0, 2 * B))))
        if trial >= 1:
            for pos in rng.integers(0, len(log), size=20):
                log[int(pos)] ^= int(rng.integers(1, 256))
        if trial >= 2:
            del log[len(log) - int(rng.integers(1, 5000)):]
        _check_scan_device(bytes(log), shift=shift)
    _check_scan_device(_oracle_encode(_random_records(rng, 50)) + bytes(3 * B + 123), shift=shift)
    _check_scan_device(rng.integers(0, 256, size=5 * B + 77, dtype=np.uint8).tobytes(), shift=shift)
    # many tiny records: long header chains within a block (> 64 records per
    # block: past wal_hist's header cache)
    _check_scan_device(_oracle_encode([bytes([k % 251]) * (k % 9) for k in range(20000)]), shift=shift)


def test_scan_device_record_edges(gpu):
    """Record-boundary cases: units of every length 0..70 around 1 KiB and 4
    KiB edges, units ending exactly on a granule / row, blocks of exactly 64 /
    65 / 128 / 200 records (wal_hist's 64-header cache and the walk past it),
    ZERO and BAD_LENGTH headers mid-block, a log ending inside a header."""
    rng = np.random.default_rng(37)
    for fill in (1000, 1017, 4090, 4096 - 7, 4096 - 6, 4096 + 3, 8181):
        recs = [bytes(fill)] + [rng.integers(0, 256, size=k, dtype=np.uint8).tobytes() for k in range(71)]
        _check_scan_device(_oracle_encode(recs))
    for per in (64, 65, 128, 200):  # records per block
        ln = (B // per) - H
        _check_scan_device(_oracle_encode([bytes([7]) * ln for _ in range(3 * per)]))
    log = bytearray(_oracle_encode(_random_records(rng, 200, maxlog=12)))
    log[5000:5007] = bytes(7)                      # a ZERO header mid-block (or inside a payload)
    log[B + 300 + 4:B + 300 + 6] = (60000).to_bytes(2, "little")  # a length past the block
    _check_scan_device(bytes(log))
    for cut in (1, 3, 6, 7, 100):
        _check_scan_device(bytes(log[:len(log) - cut]))
    big = _oracle_encode(_random_records(rng, 3000, maxlog=16))
    _check_scan_device(big)


def test_scan_device_capacity(gpu):
    """Too small a capacity: the count is reported and the caller retries."""
    rng = np.random.default_rng(31)
    log = _oracle_encode(_random_records(rng, 500))
    n = len(W.scan_log(log)[0])
    _check_scan_device(log, cap=n - 1)
    _check_scan_device(log, cap=n + 100)
    _check_scan_device(log, cap=n - 1, shift=8)
    # > 64 records per block, at and around the exact capacity
    tiny = _oracle_encode([bytes([k % 7]) * (k % 5) for k in range(30000)])
    n = len(W.scan_log(tiny)[0])
    for cap in (n - 1, n, n + 1, 2 * n):
        _check_scan_device(tiny, cap=cap)


def test_scan_device_large_logs(gpu):
    """The device scan on logs of a block per CU and more: bench-like mixed records,
    corruption, truncation, a zero tail, every block's first record a
    fragment, first records around the phase-A threshold (2,048 / 2,049-B
    units) followed by > 64 tiny records, too small a capacity, an 8-B-aligned
    log."""
    rng = np.random.default_rng(41)
    mixed = _random_records(rng, 2600, maxlog=16)
    log = bytearray(_oracle_encode(mixed, int(rng.integers(0, B))))
    assert len(log) >= 256 * B, len(log)
    _check_scan_device(bytes(log))
    _check_scan_device(bytes(log), shift=8)
    n = len(W.scan_log(bytes(log))[0])
    _check_scan_device(bytes(log), cap=n - 1)
    for pos in rng.integers(0, len(log), size=200):
        log[int(pos)] ^= int(rng.integers(1, 256))
    for blk in rng.integers(0, len(log) // B, size=10):  # first headers hit directly
        log[int(blk) * B + 4 + int(rng.integers(0, 3))] ^= 0x5a
    _check_scan_device(bytes(log[:len(log) - 777]))
    # 40 KiB records: each block's first record a FIRST / MIDDLE / LAST fragment
    frag = _oracle_encode([rng.integers(0, 256, size=40000, dtype=np.uint8).tobytes() for _ in range(260)])
    _check_scan_device(frag + bytes(2 * B + 5))
    # phase-A units around the threshold (a first record of 2,047 / 2,048 B of
    # payload: unit 2,048 / 2,049) and many tiny records per block
    edge = []
    for k in range(300):  # each group fills its block exactly: the next one's record is a first record
        grp = [bytes([k % 256]) * (2047 + k % 3)] + [bytes([k % 5]) * (k % 4)] * (3 + k % 90)
        grp.append(bytes(B - sum(H + len(r) for r in grp) - H))
        edge.extend(grp)
    elog = _oracle_encode(edge)
    assert len(elog) == 300 * B
    _check_scan_device(elog)


def test_scan_device_rejects_non_byte_views(gpu):
    """A log passed as an int32/int64 view would scan numel() < bytes; a
    workspace on another dtype is rejected too."""
    import torch

    import lvgpu
    import lvgpu.wal as LW
    log = _oracle_encode([b"abc" * 100, b"x" * 5000])
    pad = bytes(-len(log) % 8)
    d = torch.frombuffer(bytearray(log + pad), dtype=torch.uint8).to(gpu)
    for view in (d.view(torch.int32), d.view(torch.int64)):
        with pytest.raises(lvgpu.LvError):
            LW.scan_device(view, 16)
    with pytest.raises(lvgpu.LvError):
        LW.scan_device(d, 16, workspace=torch.empty(1 << 20, dtype=torch.int32, device=gpu))
