"""Replays the reference WAL test-suite (src/log_writer.rs:460-838, the
LogTest harness at :268-443) against the Python WAL restatement
(oracle/wal_oracle.py), with the reference's own expected values.  This pins
the WAL oracle the GPU verify/encode paths are checked against."""
import hashlib

import pytest

import wal_oracle as W

B, H = W.BLOCK_SIZE, W.HEADER_SIZE


class LogTest:
    """log_writer.rs:268-443."""

    def __init__(self):
        self.dest = bytearray()
        self.writer = W.Writer(self.dest)
        self.source = W.StringSource()
        self.reporter = W.ReportCollector()
        self.reading = False
        self.reader = W.Reader(self.source, self.reporter, True, 0)

    def read(self):
        if not self.reading:
            self.reading = True
            self.source.contents = bytes(self.dest)
        r = self.reader.read_record()
        return "EOF" if r is None else r.decode()

    def write(self, msg):
        assert not self.reading
        self.writer.add_record(msg.encode())

    def written_bytes(self):
        return len(self.dest)

    def dropped_bytes(self):
        return self.reporter.dropped_bytes

    def report_message(self):
        return self.reporter.message

    def reopen_for_append(self):
        self.writer = W.Writer(self.dest)

    def force_error(self):
        self.source.force_error = True

    def match_error(self, msg):
        return "OK" if msg in self.reporter.message else self.reporter.message

    def increment_bytes(self, off, delta):
        self.dest[off] = (self.dest[off] + delta) & 0xFF

    def fix_checksum(self, hoff, ln):
        c = W.mask(W.value(bytes(self.dest[hoff + 6:hoff + 7 + ln])))
        self.dest[hoff:hoff + 4] = W.encode_fixed_32(c)

    def shrink_size(self, n):
        del self.dest[len(self.dest) - n:]

    def set_byte(self, off, v):
        self.dest[off] = v

    def start_reading_at(self, off):
        self.reader = W.Reader(self.source, self.reporter, True, off)

    def write_initial_offset_log(self):
        for i in range(len(SIZES)):
            self.write(chr(ord("a") + i) * SIZES[i])

    def check_initial_offset_record(self, initial_offset, expected):
        self.write_initial_offset_log()
        self.reading = True
        self.source.contents = bytes(self.dest)
        rd = W.Reader(self.source, self.reporter, True, initial_offset)
        while expected < len(SIZES):
            rec = rd.read_record()
            assert rec is not None
            assert len(rec) == SIZES[expected]
            assert rd.last_record_offset == OFFSETS[expected]
            assert rec[0] == ord("a") + expected
            expected += 1

    def check_offset_past_end_returns_no_records(self, past):
        self.write_initial_offset_log()
        self.reading = True
        self.source.contents = bytes(self.dest)
        rd = W.Reader(self.source, self.reporter, True, self.written_bytes() + past)
        assert rd.read_record() is None


SIZES = [10000, 10000, 2 * B - 1000, 1, 13716, B - H]  # log_writer.rs:246-253
OFFSETS = [0, H + 10000, 2 * (H + 10000), 2 * (H + 10000) + (2 * B - 1000) + 3 * H,
           2 * (H + 10000) + (2 * B - 1000) + 3 * H + H + 1, 3 * B]  # :255-266


def test_empty():
    assert LogTest().read() == "EOF"


def test_read_write():
    t = LogTest()
    for m in ("foo", "bar", "", "xxxx"):
        t.write(m)
    assert t.read() == "foo"


def test_add_record_foo_header_bytes():
    t = LogTest()
    t.write("foo")
    assert bytes(t.dest[:7]).hex() == "dd5fb37a030001"


@pytest.mark.slow
def test_many_blocks():
    t = LogTest()
    for i in range(100000):
        t.write(str(i))
    for i in range(100000):
        assert t.read() == str(i)
    assert t.read() == "EOF"


def test_fragmentation():
    t = LogTest()
    t.write("small")
    t.write(W.big_string("medium", 50000))
    t.write(W.big_string("large", 100000))
    assert t.read() == "small"
    assert t.read() == W.big_string("medium", 50000)
    assert t.read() == W.big_string("large", 100000)
    assert t.read() == "EOF"


def test_marginal_trailer():
    t = LogTest()
    n = B - 2 * H
    t.write(W.big_string("foo", n))
    assert t.written_bytes() == B - H
    t.write("")
    t.write("bar")
    assert t.read() == W.big_string("foo", n)
    assert t.read() == ""
    assert t.read() == "bar"
    assert t.read() == "EOF"


def test_marginal_trailer_2():
    t = LogTest()
    n = B - 2 * H
    t.write(W.big_string("foo", n))
    assert t.written_bytes() == B - H
    t.write("bar")
    assert t.read() == W.big_string("foo", n)
    assert t.read() == "bar"
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 0
    assert t.report_message() == ""


def test_short_trailer():
    t = LogTest()
    n = B - 2 * H + 4
    t.write(W.big_string("foo", n))
    assert t.written_bytes() == B - H + 4
    t.write("")
    t.write("bar")
    assert t.read() == W.big_string("foo", n)
    assert t.read() == ""
    assert t.read() == "bar"
    assert t.read() == "EOF"


def test_aligned_eof():
    t = LogTest()
    n = B - 2 * H + 4
    t.write(W.big_string("foo", n))
    assert t.written_bytes() == B - H + 4
    assert t.read() == W.big_string("foo", n)
    assert t.read() == "EOF"


def test_open_for_append():
    t = LogTest()
    t.write("hello")
    t.reopen_for_append()
    t.write("world")
    assert t.read() == "hello"
    assert t.read() == "world"
    assert t.read() == "EOF"


def test_rand_read():
    t = LogTest()
    wr = W.Random(301)
    for i in range(500):
        t.write(W.random_skewed_string(i, wr))
    rr = W.Random(301)
    for i in range(500):
        assert t.read() == W.random_skewed_string(i, rr)
    assert t.read() == "EOF"


def test_bad_record_type():
    t = LogTest()
    t.write("foo")
    t.increment_bytes(6, 100)
    t.fix_checksum(0, 3)
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 3


def test_truncated_trailing_record_is_ignored():
    t = LogTest()
    t.write("foo")
    t.shrink_size(4)
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 0
    assert t.report_message() == ""


def test_bad_length():
    t = LogTest()
    t.write(W.big_string("bar", B - H))
    t.write("foo")
    t.increment_bytes(4, 1)
    assert t.read() == "foo"
    assert t.dropped_bytes() == B
    assert t.match_error("bad record length") == "OK"


def test_bad_length_at_end_is_ignored():
    t = LogTest()
    t.write("foo")
    t.shrink_size(1)
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 0
    assert t.report_message() == ""


def test_checksum_mismatch():
    t = LogTest()
    t.write("foo")
    t.increment_bytes(0, 10)
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 10
    assert t.match_error("checksum mismatch") == "OK"


@pytest.mark.parametrize("ty", [W.MIDDLE, W.LAST])
def test_unexpected_middle_last_type(ty):
    t = LogTest()
    t.write("foo")
    t.set_byte(6, ty)
    t.fix_checksum(0, 3)
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 3
    assert t.match_error("missing start") == "OK"


def test_unexpected_full_type():
    t = LogTest()
    t.write("foo")
    t.write("bar")
    t.set_byte(6, W.FIRST)
    t.fix_checksum(0, 3)
    assert t.read() == "bar"
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 3
    assert t.match_error("partial record without end") == "OK"


def test_unexpected_first_type():
    t = LogTest()
    t.write("foo")
    t.write(W.big_string("bar", 100000))
    t.set_byte(6, W.FIRST)
    t.fix_checksum(0, 3)
    assert t.read() == W.big_string("bar", 100000)
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 3
    assert t.match_error("partial record without end") == "OK"


def test_missing_last_is_ignored():
    t = LogTest()
    t.write(W.big_string("bar", B))
    t.shrink_size(14)
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 0
    assert t.report_message() == ""


def test_partial_last_is_ignored():
    t = LogTest()
    t.write(W.big_string("bar", B))
    t.shrink_size(1)
    assert t.read() == "EOF"
    assert t.dropped_bytes() == 0
    assert t.report_message() == ""


def test_skip_into_multi_record():
    t = LogTest()
    t.write(W.big_string("foo", 3 * B))
    t.write("correct")
    t.start_reading_at(B)
    assert t.read() == "correct"
    assert t.dropped_bytes() == 0
    assert t.report_message() == ""
    assert t.read() == "EOF"


def test_error_joins_record():
    t = LogTest()
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
def test_initial_offsets(off, exp):
    LogTest().check_initial_offset_record(off, exp)


@pytest.mark.parametrize("past", [0, 5])
def test_offset_past_end(past):
    LogTest().check_offset_past_end_returns_no_records(past)


def test_fixture_matches_oracle(wal_golden):
    """The committed WAL fixture still matches the restatement (small scenarios)."""
    for s in wal_golden["scenarios"]:
        if s["log_hex"] is not None:
            log = bytes.fromhex(s["log_hex"])
            assert hashlib.sha256(log).hexdigest() == s["log_sha256"]
            recs = W.wal_physical_records(log)
            if s["physical_records"] is not None and s["dropped_bytes"] == 0:
                assert [list(r) for r in recs] == s["physical_records"]
