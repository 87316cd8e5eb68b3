"""Replays the reference WAL test-suite (src/log_writer.rs:460-838, the
LogTest harness at :268-443) with the reference's own expected values against
three readers/writers:

  oracle  the Python restatement (oracle/wal_oracle.py) — pins the oracle;
  native  the product's host Reader (csrc/wal_host.cc, lv_wal_reader_*) fed a
          scan the oracle computed (lv_wal_scan_from_arrays) — runs on CPU;
  gpu     writes through lv_wal_encode_host (header CRCs batched on the GPU)
          and reads through lv_wal_scan_host (framing + CRCs on the GPU) and
          the host Reader.
"""
import hashlib

import pytest

import wal_oracle as W

B, H = W.BLOCK_SIZE, W.HEADER_SIZE


class LogTest:
    """log_writer.rs:268-443, over one of the backends: the oracle, the native
    reader over an oracle scan, the GPU (encode + lv_wal_scan_host), and the
    GPU with the pipelined scan (lv_wal_scan_host_pipelined)."""

    def __init__(self, backend="oracle"):
        self.backend = backend
        self.dest = bytearray()
        self.pending = []          # gpu backend: records not yet encoded
        self.writer_base = 0       # dest length when the current Writer was made
        self.writer = W.Writer(self.dest)
        self.source = W.StringSource()
        self.reporter = W.ReportCollector()
        self.reading = False
        self.initial_offset = 0
        self.reader = None
        if backend == "oracle":
            self.reader = W.Reader(self.source, self.reporter, True, 0)
        self.gpu = backend in ("gpu", "gpu_pipelined")

    # -- writer side --
    def _flush(self):
        if self.pending:
            import lvgpu.wal as LW
            # the Writer's block offset is the bytes it has written itself
            # (Writer::new_with_dest_length, log_writer.rs:48-56)
            self.dest += LW.encode(self.pending, dest_length=len(self.dest) - self.writer_base)
            self.pending = []

    def write(self, msg):
        assert not self.reading
        if self.gpu:
            self.pending.append(msg.encode())
        else:
            self.writer.add_record(msg.encode())

    def reopen_for_append(self):  # log_writer.rs:326-329: Writer::new, block offset 0
        self._flush()
        self.writer = W.Writer(self.dest)
        self.writer_base = len(self.dest)

    # -- reader side --
    def _native_reader(self, log, initial_offset):
        import lvgpu.wal as LW
        if self.backend == "gpu":
            scan = LW.Scan.host(log)
        elif self.backend == "gpu_pipelined":  # the reader waits on the scan's chunks as it goes
            scan = LW.Scan.host_pipelined(log)
        else:
            scan = LW.Scan.from_arrays(*W.scan_log(log))
        return LW.Reader(log, scan, self.reporter, True, initial_offset)

    def _start(self):
        self._flush()
        self.reading = True
        self.source.contents = bytes(self.dest)
        if self.backend != "oracle":
            self.reader = self._native_reader(self.source.contents, self.initial_offset)

    def read(self):
        if not self.reading:
            self._start()
        r = self.reader.read_record()
        return "EOF" if r is None else r.decode()

    def last_record_offset(self, rd):
        return rd.last_record_offset if self.backend == "oracle" else rd.last_record_offset()

    def written_bytes(self):
        self._flush()
        return len(self.dest)

    def dropped_bytes(self):
        return self.reporter.dropped_bytes

    def report_message(self):
        return self.reporter.message

    def match_error(self, msg):
        return "OK" if msg in self.reporter.message else self.reporter.message

    def increment_bytes(self, off, delta):
        self._flush()
        self.dest[off] = (self.dest[off] + delta) & 0xFF

    def fix_checksum(self, hoff, ln):
        self._flush()
        c = W.mask(W.value(bytes(self.dest[hoff + 6:hoff + 7 + ln])))
        self.dest[hoff:hoff + 4] = W.encode_fixed_32(c)

    def shrink_size(self, n):
        self._flush()
        del self.dest[len(self.dest) - n:]

    def set_byte(self, off, v):
        self._flush()
        self.dest[off] = v

    def start_reading_at(self, off):
        if self.backend == "oracle":
            self.reader = W.Reader(self.source, self.reporter, True, off)
        else:
            self.initial_offset = off

    def _reader_at(self, off):
        self._flush()
        self.reading = True
        self.source.contents = bytes(self.dest)
        if self.backend == "oracle":
            return W.Reader(self.source, self.reporter, True, off)
        return self._native_reader(self.source.contents, off)

    def write_initial_offset_log(self):
        for i in range(len(SIZES)):
            self.write(chr(ord("a") + i) * SIZES[i])

    def check_initial_offset_record(self, initial_offset, expected):
        self.write_initial_offset_log()
        rd = self._reader_at(initial_offset)
        while expected < len(SIZES):
            rec = rd.read_record()
            assert rec is not None
            assert len(rec) == SIZES[expected]
            assert self.last_record_offset(rd) == OFFSETS[expected]
            assert rec[0] == ord("a") + expected
            expected += 1

    def check_offset_past_end_returns_no_records(self, past):
        self.write_initial_offset_log()
        rd = self._reader_at(self.written_bytes() + past)
        assert rd.read_record() is None


@pytest.fixture(params=["oracle", "native", pytest.param("gpu", marks=pytest.mark.gpu),
                        pytest.param("gpu_pipelined", marks=pytest.mark.gpu)])
def LogTest_(request):
    if request.param in ("gpu", "gpu_pipelined"):
        request.getfixturevalue("gpu")
    return lambda: LogTest(request.param)


SIZES = [10000, 10000, 2 * B - 1000, 1, 13716, B - H]  # log_writer.rs:246-253
OFFSETS = [0, H + 10000, 2 * (H + 10000), 2 * (H + 10000) + (2 * B - 1000) + 3 * H,
           2 * (H + 10000) + (2 * B - 1000) + 3 * H + H + 1, 3 * B]  # :255-266


def test_empty(LogTest_):
    assert LogTest_().read() == "EOF"


def test_read_write(LogTest_):
    t = LogTest_()
    for m in ("foo", "bar", "", "xxxx"):
        t.write(m)
    assert t.read() == "foo"


def test_add_record_foo_header_bytes(LogTest_):
    t = LogTest_()
    t.write("foo")
    assert t.written_bytes() == 10
    assert bytes(t.dest[:7]).hex() == "dd5fb37a030001"


@pytest.mark.slow
def test_many_blocks(LogTest_):
    t = LogTest_()
    for i in range(100000):
        t.write(str(i))
    for i in range(100000):
        assert t.read() == str(i)
    assert t.read() == "EOF"


def test_fragmentation(LogTest_):
    t = LogTest_()
    t.write("small")
    t.write(W.big_string("medium", 50000))
    t.write(W.big_string("large", 100000))
    assert t.read() == "small"
    assert t.read() == W.big_string("medium", 50000)
    assert t.read() == W.big_string("large", 100000)
    assert t.read() == "EOF"


def test_marginal_trailer(LogTest_):
    t = LogTest_()
    n = B - 2 * H
    t.write(W.big_string("foo", n))
    assert t.written_bytes() == B - H
    t.write("")
    t.write("bar")
    assert t.read() == W.big_string("foo", n)
    assert t.read() == ""
    assert t.read() == "bar"
    assert t.read() == "EOF"


def test_marginal_trailer_2(LogTest_):
    t = LogTest_()
    n = B - 2 * H
    t.write(W.big_string("foo", n))
    assert t.written_bytes() == B - H
    t.write("bar")
    assert t.read() == W.big_string("foo", n)
    assert t.read() == "bar"
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 0
    assert t.report_message() == ""


def test_short_trailer(LogTest_):
    t = LogTest_()
    n = B - 2 * H + 4
    t.write(W.big_string("foo", n))
    assert t.written_bytes() == B - H + 4
    t.write("")
    t.write("bar")
    assert t.read() == W.big_string("foo", n)
    assert t.read() == ""
    assert t.read() == "bar"
    assert t.read() == "EOF"


def test_aligned_eof(LogTest_):
    t = LogTest_()
    n = B - 2 * H + 4
    t.write(W.big_string("foo", n))
    assert t.written_bytes() == B - H + 4
    assert t.read() == W.big_string("foo", n)
    assert t.read() == "EOF"


def test_open_for_append(LogTest_):
    t = LogTest_()
    t.write("hello")
    t.reopen_for_append()
    t.write("world")
    assert t.read() == "hello"
    assert t.read() == "world"
    assert t.read() == "EOF"


def test_rand_read(LogTest_):
    t = LogTest_()
    wr = W.Random(301)
    for i in range(500):
        t.write(W.random_skewed_string(i, wr))
    rr = W.Random(301)
    for i in range(500):
        assert t.read() == W.random_skewed_string(i, rr)
    assert t.read() == "EOF"


def test_bad_record_type(LogTest_):
    t = LogTest_()
    t.write("foo")
    t.increment_bytes(6, 100)
    t.fix_checksum(0, 3)
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 3


def test_truncated_trailing_record_is_ignored(LogTest_):
    t = LogTest_()
    t.write("foo")
    t.shrink_size(4)
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 0
    assert t.report_message() == ""


def test_bad_length(LogTest_):
    t = LogTest_()
    t.write(W.big_string("bar", B - H))
    t.write("foo")
    t.increment_bytes(4, 1)
    assert t.read() == "foo"
    assert t.dropped_bytes() == B
    assert t.match_error("bad record length") == "OK"


def test_bad_length_at_end_is_ignored(LogTest_):
    t = LogTest_()
    t.write("foo")
    t.shrink_size(1)
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 0
    assert t.report_message() == ""


def test_checksum_mismatch(LogTest_):
    t = LogTest_()
    t.write("foo")
    t.increment_bytes(0, 10)
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 10
    assert t.match_error("checksum mismatch") == "OK"


@pytest.mark.parametrize("ty", [W.MIDDLE, W.LAST])
def test_unexpected_middle_last_type(LogTest_, ty):
    t = LogTest_()
    t.write("foo")
    t.set_byte(6, ty)
    t.fix_checksum(0, 3)
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 3
    assert t.match_error("missing start") == "OK"


def test_unexpected_full_type(LogTest_):
    t = LogTest_()
    t.write("foo")
    t.write("bar")
    t.set_byte(6, W.FIRST)
    t.fix_checksum(0, 3)
    assert t.read() == "bar"
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 3
    assert t.match_error("partial record without end") == "OK"


def test_unexpected_first_type(LogTest_):
    t = LogTest_()
    t.write("foo")
    t.write(W.big_string("bar", 100000))
    t.set_byte(6, W.FIRST)
    t.fix_checksum(0, 3)
    assert t.read() == W.big_string("bar", 100000)
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 3
    assert t.match_error("partial record without end") == "OK"


def test_missing_last_is_ignored(LogTest_):
    t = LogTest_()
    t.write(W.big_string("bar", B))
    t.shrink_size(14)
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 0
    assert t.report_message() == ""


def test_partial_last_is_ignored(LogTest_):
    t = LogTest_()
    t.write(W.big_string("bar", B))
    t.shrink_size(1)
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 0
    assert t.report_message() == ""


def test_skip_into_multi_record(LogTest_):
    t = LogTest_()
    t.write(W.big_string("foo", 3 * B))
    t.write("correct")
    t.start_reading_at(B)
    assert t.read() == "correct"
    assert t.dropped_bytes() == 0
    assert t.report_message() == ""
    assert t.read() == "EOF"


def test_error_joins_record(LogTest_):
    t = LogTest_()
    t.write(W.big_string("foo", B))
    t.write(W.big_string("bar", B))
    t.write("correct")
    for o in range(B, 2 * B):
        t.set_byte(o, ord("x"))
    assert t.read() == "correct"
    assert t.read() == "EOF"
    assert 2 * B <= t.dropped_bytes() <= 2 * B + 100


@pytest.mark.parametrize("off,exp", [
    (0, 0), (1, 1), (10000, 1), (10007, 1), (10008, 2), (20014, 2), (20015, 3),
    (B - 4, 3), (B + 1, 3), (2 * B + 1, 3),
    (2 * (H + 10000) + (2 * B - 1000) + 3 * H, 3), (3 * B - 3, 5)])
def test_initial_offsets(LogTest_, off, exp):
    LogTest_().check_initial_offset_record(off, exp)


@pytest.mark.parametrize("past", [0, 5])
def test_offset_past_end(LogTest_, past):
    LogTest_().check_offset_past_end_returns_no_records(past)


def test_fixture_matches_oracle(wal_golden):
    """The committed WAL fixture still matches the restatement (small scenarios)."""
    for s in wal_golden["scenarios"]:
        if s["log_hex"] is not None:
            log = bytes.fromhex(s["log_hex"])
            assert hashlib.sha256(log).hexdigest() == s["log_sha256"]
            recs = W.wal_physical_records(log)
            if s["physical_records"] is not None and s["dropped_bytes"] == 0:
                assert [list(r) for r in recs] == s["physical_records"]
