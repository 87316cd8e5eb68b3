"""Regenerate the golden fixtures in tests/golden/ from the CPU oracle.

Run from the repo root after `make -C oracle`:

    python tests/golden/make_golden.py

Outputs (all data — inputs and expected outputs, no reference source):
  crc32c_kat.json   reference KATs (crc32c.rs:147-193) + survey vectors +
                    seeded random (offset, length, seed) cases over a
                    splitmix64 arena, each cross-checked sw == hw == bitwise.
  wal_scenarios.json  the reference LogTest WAL scenarios (log_writer.rs:460-838)
                    replayed through oracle/wal_oracle.py: log bytes digest,
                    every physical record's CRC unit and the reader outcome.
  hash_kat.json     reference hash KATs (util/hash.rs:58-75) + seeded random
                    (offset, length, seed) cases over the same arena.
  table_format.json BlockHandle / Footer encodings (table/format.rs:107-147),
                    varint cases (coding.rs:481-510) and block trailers over
                    arena slices (trailer layout parity unpinned, see
                    oracle/table_oracle.py).
"""
import ctypes
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import wal_oracle as W  # noqa: E402

ARENA_SEED = 0x4C5647505531  # "LVGPU1"
ARENA_BYTES = 1 << 20


def arena_bytes(nbytes=ARENA_BYTES, seed=ARENA_SEED):
    buf = ctypes.create_string_buffer(nbytes)
    W.lib().oracle_fill_splitmix(buf, 0, nbytes, seed)
    return buf.raw


def crc_all(seed, data):
    L = W.lib()
    a = L.oracle_extend_sw(seed, data, len(data))
    b = L.oracle_extend_hw(seed, data, len(data))
    c = L.oracle_extend_bitwise(seed, data, len(data))
    assert a == b == c, (a, b, c)
    return a


def kat_fixture():
    iscsi = bytes([
        0x01, 0xc0, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
        0x00, 0x00, 0x00, 0x14, 0x00, 0x00, 0x00, 0x00, 0x00, 0x04, 0x00, 0x00, 0x00,
        0x00, 0x14, 0x00, 0x00, 0x00, 0x18, 0x28, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
        0x00, 0x02, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00])
    ref_kats = [  # crc32c.rs:147-171, expected values from the reference test
        ("32 x 0x00", bytes(32), 0x8a9136aa),
        ("32 x 0xff", b"\xff" * 32, 0x62a8ab43),
        ("bytes 0..31", bytes(range(32)), 0x46dd794e),
        ("bytes 31..0", bytes(range(31, -1, -1)), 0x113fdb5c),
        ("48-byte iSCSI read PDU", iscsi, 0xd9963a56),
    ]
    extra = [  # SURVEY.md §8c (two independent implementations, session-verified)
        ("123456789 (standard CRC-32C check)", b"123456789", 0xe3069283),
        ("foo", b"foo", 0xcfc4ae1d),
        ("x * 256", b"x" * 256, 0x4ec8df3a),
        ("x * 1024", b"x" * 1024, 0xeb7355d9),
        ("x * 4096", b"x" * 4096, 0xa46ab21f),
        ("x * 60056", b"x" * 60056, 0xab0b73b0),
        ("x * 65536", b"x" * 65536, 0x165c0103),
        ("empty", b"", 0x00000000),
    ]
    kats = []
    for src, items in (("reference crc32c.rs:147-171", ref_kats), ("SURVEY.md 8c", extra)):
        for name, data, want in items:
            got = crc_all(0, data)
            assert got == want, (name, hex(got), hex(want))
            kats.append({"name": name, "source": src, "hex": data.hex() if len(data) <= 64 else None,
                         "fill": None if len(data) <= 64 else {"byte": data[0], "n": len(data)},
                         "value": want, "masked": W.mask(want)})
    props = {  # crc32c.rs:174-193
        "values_ne": [W.value(b"a"), W.value(b"foo")],
        "extend": {"whole": W.value(b"hello world"), "split": W.extend(W.value(b"hello "), b"world")},
        "mask_of_foo": W.mask(W.value(b"foo")),
        "mask_delta": 0xa282ead8,
        "type_crc": [W.value(bytes([t])) for t in range(5)],  # log_writer.rs:136-142
        "extend_empty_seed": {"seed": 0x12345678, "value": W.extend(0x12345678, b"")},
    }
    assert props["extend"]["whole"] == props["extend"]["split"]

    arena = arena_bytes()
    rng = random.Random(20261015)
    cases = []
    lengths = list(range(0, 80)) + [
        127, 128, 129, 255, 256, 257, 511, 512, 513, 1000, 1023, 1024, 1025, 1031,
        2047, 2048, 2049, 4095, 4096, 4097, 8191, 8192, 8193, 16383, 16384, 16385,
        32761, 32762, 32768, 60056, 65535, 65536, 65537, 70000]
    lengths += [rng.randrange(0, 70001) for _ in range(300)]
    lengths += [rng.randrange(0, 300) for _ in range(200)]
    for ln in lengths:
        for _ in range(2):
            off = rng.randrange(0, ARENA_BYTES - ln + 1)
            seed = rng.choice([0, 0xFFFFFFFF, rng.getrandbits(32)] + props["type_crc"])
            v = crc_all(seed, arena[off:off + ln])
            cases.append([off, ln, seed, v, W.mask(v)])
    return {
        "generator": "tests/golden/make_golden.py",
        "arena": {"kind": "splitmix64", "seed": ARENA_SEED, "bytes": ARENA_BYTES,
                  "rule": "byte k = byte (k & 7) of splitmix64(seed ^ (k >> 3))",
                  "sha256": hashlib.sha256(arena).hexdigest()},
        "kats": kats,
        "properties": props,
        "cases_fields": ["offset", "length", "seed", "crc", "masked_crc"],
        "cases": cases,
    }


def wal_scenarios():
    """Replays the reference LogTest scenarios (log_writer.rs:460-838) that
    exercise the CRC path, recording the bytes the writer produced and every
    CRC unit `[type || payload]` (log_reader.rs:336) the reader checked."""
    B, H = W.BLOCK_SIZE, W.HEADER_SIZE
    scen = []

    def run(name, writes, mutate=None, reads=None, initial_offset=0, ref=""):
        dest = bytearray()
        wr = W.Writer(dest)
        for w in writes:
            wr.add_record(w.encode() if isinstance(w, str) else w)
        if mutate:
            mutate(dest)
        rep = W.ReportCollector()
        rd = W.Reader(W.StringSource(bytes(dest)), rep, True, initial_offset)
        got = []
        while True:
            r = rd.read_record()
            if r is None:
                break
            got.append(r)
        units = [[len(u), W.value(u), exp] for u, exp in rd.crc_calls]
        packed = b"".join(ln.to_bytes(4, "little") + c.to_bytes(4, "little") for ln, c, _ in units)
        recs = W.wal_physical_records(bytes(dest))
        small = len(units) <= 600
        scen.append({
            "name": name, "ref": ref,
            "log_len": len(dest), "log_sha256": hashlib.sha256(bytes(dest)).hexdigest(),
            "log_hex": bytes(dest).hex() if len(dest) <= 256 else None,
            "n_reads": len(got),
            "reads_sha256": [hashlib.sha256(r).hexdigest()[:16] for r in got] if len(got) <= 600 else None,
            "reads_digest": hashlib.sha256(b"".join(len(r).to_bytes(4, "little") + r for r in got)).hexdigest(),
            "dropped_bytes": rep.dropped_bytes, "report_message": rep.message,
            "n_physical_records": len(recs),
            "physical_records": [[o, ln, t] for (o, ln, t) in recs] if small else None,
            "n_crc_units": len(units),
            "crc_units_fields": ["length", "value([type||payload])", "unmask(header crc)"],
            "crc_units": units if small else None,
            "crc_units_sha256": hashlib.sha256(packed).hexdigest(),
        })

    def inc(off, d):
        def f(buf):
            buf[off] = (buf[off] + d) & 0xFF
        return f

    def setb(off, v):
        def f(buf):
            buf[off] = v
        return f

    def fix_checksum(hoff, ln):  # log_writer.rs:347-353
        def f(buf):
            c = W.mask(W.value(bytes(buf[hoff + 6:hoff + 7 + ln])))
            buf[hoff:hoff + 4] = W.encode_fixed_32(c)
        return f

    def chain(*fs):
        def f(buf):
            for g in fs:
                g(buf)
        return f

    def shrink(n):
        def f(buf):
            del buf[len(buf) - n:]
        return f

    run("read_write", ["foo", "bar", "", "xxxx"], ref="log_writer.rs:467-475")
    run("add_record_foo", ["foo"], ref="SURVEY 8c header dd5fb37a 0300 01")
    run("many_blocks", [str(i) for i in range(100000)], ref="log_writer.rs:477-486")
    run("fragmentation", ["small", W.big_string("medium", 50000), W.big_string("large", 100000)],
        ref="log_writer.rs:489-498")
    run("marginal_trailer", [W.big_string("foo", B - 2 * H), "", "bar"], ref="log_writer.rs:501-513")
    run("short_trailer", [W.big_string("foo", B - 2 * H + 4), "", "bar"], ref="log_writer.rs:529-541")
    rnd = W.Random(301)
    run("rand_read", [W.random_skewed_string(i, rnd) for i in range(500)], ref="log_writer.rs:564-576")
    run("bad_record_type", ["foo"], chain(inc(6, 100), fix_checksum(0, 3)), ref="log_writer.rs:594-601")
    run("checksum_mismatch", ["foo"], inc(0, 10), ref="log_writer.rs:636-643")
    run("unexpected_middle_type", ["foo"], chain(setb(6, W.MIDDLE), fix_checksum(0, 3)),
        ref="log_writer.rs:645-653")
    run("unexpected_full_type", ["foo", "bar"], chain(setb(6, W.FIRST), fix_checksum(0, 3)),
        ref="log_writer.rs:665-675")
    run("bad_length", [W.big_string("bar", B - H), "foo"], inc(4, 1), ref="log_writer.rs:612-621")
    run("truncated_trailing_record_is_ignored", ["foo"], shrink(4), ref="log_writer.rs:603-610")

    def wipe_middle(buf):
        for o in range(B, 2 * B):
            buf[o] = ord("x")
    run("error_joins_record", [W.big_string("foo", B), W.big_string("bar", B), "correct"], wipe_middle,
        ref="log_writer.rs:727-750")
    return {"generator": "tests/golden/make_golden.py", "scenarios": scen}


def hash_fixture():
    L = W.lib()
    L.oracle_hash.restype = ctypes.c_uint32
    L.oracle_hash.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32]
    d5 = bytes([0x01, 0xc0] + [0] * 14 + [0x14, 0, 0, 0, 0, 0, 0x04, 0, 0, 0, 0, 0x14, 0, 0, 0, 0x18, 0x28]
               + [0] * 7 + [0x02] + [0] * 7)
    ref = [  # hash.rs:58-75, expected values from the reference test
        ("empty", b"", 0xbc9f1d34, 0xbc9f1d34),
        ("62", b"\x62", 0xbc9f1d34, 0xef1345c4),
        ("c3 97", b"\xc3\x97", 0xbc9f1d34, 0x5b663814),
        ("e2 99 a5", b"\xe2\x99\xa5", 0xbc9f1d34, 0x323c078f),
        ("e1 80 b9 32", b"\xe1\x80\xb9\x32", 0xbc9f1d34, 0xed21633a),
        ("48-byte data5", d5, 0x12345678, 0xf333dabb),
    ]
    kats = []
    for name, data, seed, want in ref:
        got = L.oracle_hash(data, len(data), seed)
        assert got == want, (name, hex(got))
        kats.append({"name": name, "hex": data.hex(), "seed": seed, "hash": want, "ref": "hash.rs:58-75"})
    arena = arena_bytes()
    rng = random.Random(0x4C564853)
    cases = []
    for i in range(800):
        ln = rng.choice([rng.randrange(0, 17), rng.randrange(0, 129), rng.randrange(0, 8193)])
        off = rng.randrange(0, ARENA_BYTES - ln + 1)
        seed = rng.choice([0, 0xbc9f1d34, rng.getrandbits(32)])
        cases.append([off, ln, seed, L.oracle_hash(arena[off:off + ln], ln, seed)])
    return {"generator": "tests/golden/make_golden.py",
            "arena": {"bytes": ARENA_BYTES, "seed": ARENA_SEED}, "kats": kats,
            "cases_fields": ["offset", "length", "seed", "hash"], "cases": cases}


def table_fixture():
    import table_oracle as T
    out = {"generator": "tests/golden/make_golden.py"}
    b = bytearray()
    T.BlockHandle(10, 20).encode_to(b)  # format.rs:107-123
    out["block_handles"] = [{"offset": 10, "size": 20, "hex": bytes(b).hex(), "ref": "format.rs:107-123"}]
    rng = random.Random(0x4C565442)
    for _ in range(40):
        o, sz = rng.getrandbits(rng.randrange(1, 65)), rng.getrandbits(rng.randrange(1, 65))
        b = bytearray()
        T.BlockHandle(o, sz).encode_to(b)
        out["block_handles"].append({"offset": o, "size": sz, "hex": bytes(b).hex()})
    f = bytearray()
    T.Footer(T.BlockHandle(50, 100), T.BlockHandle(200, 400)).encode_to(f)  # format.rs:125-147
    out["footers"] = [{"metaindex": [50, 100], "index": [200, 400], "hex": bytes(f).hex(), "ref": "format.rs:125-147"}]
    big = bytearray()
    T.Footer(T.BlockHandle(2**64 - 1, 2**64 - 1), T.BlockHandle(2**63, 1)).encode_to(big)
    out["footers"].append({"metaindex": [2**64 - 1, 2**64 - 1], "index": [2**63, 1], "hex": bytes(big).hex()})
    out["varints"] = [[v, T.encode_varint_64(v).hex()] for v in
                      [0, 1, 127, 128, 1000, 16383, 16384, 1 << 60, 2**64 - 1]]  # coding.rs:481-510
    arena = arena_bytes()
    tr = []
    for _ in range(60):
        ln = rng.choice([0, 1, rng.randrange(0, 4097), rng.randrange(0, 70000)])
        off = rng.randrange(0, ARENA_BYTES - ln + 1)
        ctype = rng.choice([0, 1])
        tr.append([off, ln, ctype, T.block_trailer(arena[off:off + ln], ctype).hex()])
    out["trailers_fields"] = ["offset", "size", "type", "trailer_hex"]
    out["trailers"] = tr
    out["trailers_note"] = "type || LE32(mask(crc32c(contents || type))); parity unpinned beyond crc32c KATs"
    return out


def main():
    with open(os.path.join(HERE, "hash_kat.json"), "w") as f:
        json.dump(hash_fixture(), f, indent=0, separators=(",", ":"))
    with open(os.path.join(HERE, "table_format.json"), "w") as f:
        json.dump(table_fixture(), f, indent=0, separators=(",", ":"))
    kat = kat_fixture()
    with open(os.path.join(HERE, "crc32c_kat.json"), "w") as f:
        json.dump(kat, f, indent=0, separators=(",", ":"))
    wal = wal_scenarios()
    with open(os.path.join(HERE, "wal_scenarios.json"), "w") as f:
        json.dump(wal, f, indent=0, separators=(",", ":"))
    print("cases", len(kat["cases"]), "scenarios", len(wal["scenarios"]))


if __name__ == "__main__":
    main()
