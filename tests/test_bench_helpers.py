"""bench.py's pure helpers (no GPU): the hash line's rooflines and the
kernel-name classification its VALU pass uses."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("lvgpu_bench", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_hash_api_of_kernel_names():
    """Every hash_kernel<Meta> variant's parameter list holds "unsigned int";
    only the template argument tells the APIs apart (rocprofv3 names)."""
    b = _bench()
    sig = "(unsigned char const*, {m}, unsigned int*, unsigned int, unsigned int)"
    assert b.hash_api_of("void lvh::hash_kernel<lvh::OffsetsMeta>" + sig.format(m="lvh::OffsetsMeta")) == "offsets"
    m32 = "lvh::PackedMeta<unsigned int>"
    assert b.hash_api_of(f"void lvh::hash_kernel<{m32}>" + sig.format(m=m32)) == "packed_u32"
    m64 = "lvh::PackedMeta<unsigned long>"
    assert b.hash_api_of(f"void lvh::hash_kernel<{m64}>" + sig.format(m=m64)) == "packed_u64"


def test_hash_rooflines_pick_the_binding_bound():
    b = _bench()
    key, moved, ms = 600_000_000, 870_000_000, 0.14
    roof, hbm, valu = b.hash_rooflines(key, ms, None, moved)
    assert roof is hbm and valu is None and roof["bound"] == "hbm"
    assert abs(hbm["frac"] - key / (ms * 1e-3) / 8e12) < 1e-3
    assert abs(hbm["frac_all_bytes"] - moved / (ms * 1e-3) / 8e12) < 1e-3
    # a VALU count far below the issue rate: HBM binds
    roof, hbm, valu = b.hash_rooflines(key, ms, 1e6, moved)
    assert roof is hbm and valu["frac"] < hbm["frac"]
    # the rule compares the reported numbers: a VALU frac between
    # the key-byte and all-byte HBM fracs makes VALU the roofline
    peak = b.VALU_SIMDS * b.VALU_CLOCK_HZ / b.VALU_CYCLES * ms * 1e-3
    mid = (hbm["frac"] + hbm["frac_all_bytes"]) / 2
    roof, hbm, valu = b.hash_rooflines(key, ms, mid * peak, moved)
    assert roof is valu and hbm["frac"] < valu["frac"] < hbm["frac_all_bytes"]
    # one at the issue peak: VALU binds
    peak = b.VALU_SIMDS * b.VALU_CLOCK_HZ / b.VALU_CYCLES * ms * 1e-3
    roof, hbm, valu = b.hash_rooflines(key, ms, peak, moved)
    assert roof is valu and abs(valu["frac"] - 1.0) < 1e-3


def test_read_pmc_per_kernel(tmp_path):
    """The --wal-device traffic pass: per-kernel means of one counter, fill
    kernels and other counters ignored, FETCH_SIZE doubled (gfx950)."""
    b = _bench()
    rows = ["Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value",
            '1,"void lvk::wal_hist(unsigned char const*, unsigned long)",FETCH_SIZE,100',
            '5,"void lvk::wal_hist(unsigned char const*, unsigned long)",FETCH_SIZE,300',
            '2,"void lvk::wal_scatter(unsigned char const*)",FETCH_SIZE,50',
            '3,"void lvk::fill_bytes(unsigned char*)",FETCH_SIZE,999',
            '4,"void lvk::wal_scatter(unsigned char const*)",WRITE_SIZE,7']
    p = tmp_path / "c.csv"
    p.write_text("\n".join(rows) + "\n")
    assert b.read_pmc_per_kernel(str(p), "FETCH_SIZE") == {"lvk::wal_hist": 2.0 * 1024 * 200,
                                                           "lvk::wal_scatter": 2.0 * 1024 * 50}
    assert b.read_pmc_per_kernel(str(p), "WRITE_SIZE") == {"lvk::wal_scatter": 7.0 * 1024}
    # keep / last: the named kernels' last launches only
    assert b.read_pmc_per_kernel(str(p), "FETCH_SIZE", {"lvk::wal_hist"}, 1) == {"lvk::wal_hist": 2.0 * 1024 * 300}


def test_wal_units_typed_match_the_oracle_writer():
    """bench.py --variants' C2 writer case: fragment lengths and record types
    of the first physical records equal what the oracle Writer
    (log_writer.rs:62-110) lays out for the same Random(301).skewed(17)
    records, and the header CRC is mask(extend(type_crc[t], fragment))."""
    import sys
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import wal_oracle as W
    b = _bench()
    m = 1500
    u, t = b.wal_units_typed(m)
    r, log = W.Random(301), bytearray()
    w = W.Writer(log)
    while True:
        w.add_record(bytes(r.skewed(17)))
        if len(log) > int(u.sum()) + 7 * m:
            break
    phys = W.wal_physical_records(bytes(log))[:m]
    assert np.array_equal(np.array([p[1] for p in phys]), u)
    assert np.array_equal(np.array([p[2] for p in phys]), t)
    tc = [W.value(bytes([k])) for k in range(5)]
    for o, ln, ty in phys[:200]:
        assert W.decode_fixed_32(bytes(log[o:o + 4])) == W.mask(W.extend(tc[ty], bytes(log[o + 7:o + 7 + ln])))


def test_parse_cpulist():
    """bench.py --wal's placement reads the GPU's local_cpulist."""
    b = _bench()
    assert b.parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert b.parse_cpulist("64-127,192-255") == set(range(64, 128)) | set(range(192, 256))
    assert b.parse_cpulist("") == set()
