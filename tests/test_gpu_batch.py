"""GPU parity: the HIP batch kernels (through the C ABI) against the CPU oracle
(restating crc32c.rs) — bit-exact, on the reference KATs, the committed golden
cases, edge cases (empty, < 4 bytes, every start alignment, ragged tails,
max WAL fragment, 64 KiB+), every kernel group size, masked and seeded
outputs, and the full-size configuration (262,144 x 4 KiB = 1 GiB)."""
import ctypes
import random

import numpy as np
import pytest

from conftest import kat_bytes
import lvgpu
import wal_oracle as W

pytestmark = pytest.mark.gpu

GROUPS = [1, 4, 16, 64]


def oracle_batch(arena: bytes, off, ln, seed, masked):
    L = W.lib()
    a = np.frombuffer(arena, dtype=np.uint8)
    o = np.ascontiguousarray(off, dtype=np.uint64)
    n = np.ascontiguousarray(ln, dtype=np.uint32)
    s = None if seed is None else np.ascontiguousarray(seed, dtype=np.uint32)
    out = np.zeros(o.size, dtype=np.uint32)
    L.oracle_batch(a.ctypes.data, o.ctypes.data, n.ctypes.data, None if s is None else s.ctypes.data,
                   out.ctypes.data, o.size, 1 if masked else 0)
    return out


def gpu_batch(torch, dev, arena: bytes, off, ln, seed, masked, group=None):
    a = torch.frombuffer(bytearray(arena), dtype=torch.uint8).to(dev)
    o = torch.from_numpy(np.ascontiguousarray(off, dtype=np.int64)).to(dev)
    n = torch.from_numpy(np.ascontiguousarray(ln, dtype=np.uint32).view(np.int32)).to(dev)
    s = None if seed is None else torch.from_numpy(np.ascontiguousarray(seed, dtype=np.uint32).view(np.int32)).to(dev)
    out = lvgpu.batch(a, o, n, s, masked=masked, group=group)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


@pytest.fixture(scope="module")
def torch_dev(gpu):
    import torch
    return torch, gpu


@pytest.mark.parametrize("group", [None] + GROUPS)
def test_kats_every_alignment(torch_dev, kat, group):
    torch, dev = torch_dev
    pieces, offs, lens, want = bytearray(), [], [], []
    for k in kat["kats"]:
        d = kat_bytes(k)
        for shift in range(16):
            pieces += bytes(shift)
            offs.append(len(pieces))
            lens.append(len(d))
            pieces += d
            want.append(k["value"])
    got = gpu_batch(torch, dev, bytes(pieces), offs, lens, None, False, group)
    assert list(got) == want


@pytest.mark.parametrize("group", [None] + GROUPS)
@pytest.mark.parametrize("masked", [False, True])
def test_golden_cases(torch_dev, kat, arena, group, masked):
    torch, dev = torch_dev
    c = np.array(kat["cases"], dtype=np.uint64)
    got = gpu_batch(torch, dev, arena, c[:, 0], c[:, 1], c[:, 2], masked, group)
    want = c[:, 4] if masked else c[:, 3]
    bad = np.nonzero(got != want.astype(np.uint32))[0]
    assert bad.size == 0, [(int(c[i, 0]), int(c[i, 1]), hex(int(got[i])), hex(int(want[i]))) for i in bad[:10]]


@pytest.mark.parametrize("group", [None] + GROUPS)
def test_small_lengths_all_offsets(torch_dev, arena, group):
    """Every length 0..300 at every start offset mod 64, random seeds."""
    torch, dev = torch_dev
    rng = random.Random(11 + (group or 0))
    offs, lens, seeds = [], [], []
    for ln in range(0, 301):
        for mis in range(0, 64, 3):
            offs.append(4096 * rng.randrange(1, 200) + mis)
            lens.append(ln)
            seeds.append(rng.getrandbits(32))
    want = oracle_batch(arena, offs, lens, seeds, False)
    got = gpu_batch(torch, dev, arena, offs, lens, seeds, False, group)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(offs[i], lens[i]) for i in bad[:10]]


@pytest.mark.parametrize("group", GROUPS)
@pytest.mark.parametrize("block_len", [1, 3, 4, 5, 15, 16, 17, 100, 128, 129, 1000, 1024, 1025, 4096,
                                       4100, 16384, 16385, 32762, 65536, 70001])
def test_strided_blocks(torch_dev, group, block_len):
    torch, dev = torch_dev
    rng = np.random.default_rng(block_len)
    n = max(8, min(600, (4 << 20) // max(block_len, 1)))
    stride = block_len + int(rng.integers(0, 40))
    total = stride * n + 64
    host = rng.integers(0, 256, size=total, dtype=np.uint8).tobytes()
    seeds = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    base_off = int(rng.integers(0, 16))
    offs = base_off + np.arange(n, dtype=np.uint64) * stride
    want = oracle_batch(host, offs, np.full(n, block_len, np.uint32), seeds, True)
    t = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(dev)
    sd = torch.from_numpy(seeds.view(np.int32)).to(dev)
    out = lvgpu.batch_strided(t[base_off:], stride, block_len, n, seed=sd, masked=True, group=group)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    assert np.array_equal(got, want)


def test_mixed_lengths_zipf(torch_dev):
    """Config-4 shape (Zipf 32 B - 64 KiB, misaligned), reduced count."""
    torch, dev = torch_dev
    rng = np.random.default_rng(0xC0FFEE)
    k = np.minimum(rng.zipf(1.1, size=20000), 2048)
    lens = (32 * k - rng.integers(0, 32, size=k.size)).astype(np.uint32)
    offs = np.zeros(lens.size, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    total = int(offs[-1] + lens[-1]) + 16
    host = bytearray(total)
    W.lib().oracle_fill_splitmix(ctypes.addressof(ctypes.c_char.from_buffer(host)), 0, total, 77)
    host = bytes(host)
    want = oracle_batch(host, offs, lens, None, False)
    got = gpu_batch(torch, dev, host, offs, lens, None, False)
    assert np.array_equal(got, want)


def test_wal_units(torch_dev, wal_golden):
    """Batched form of log_reader.rs:335-336 over the WAL fixtures' CRC units:
    value([type||payload]) of every physical record of the fragmentation scenario."""
    torch, dev = torch_dev
    dest = bytearray()
    wr = W.Writer(dest)
    for m in ("small", W.big_string("medium", 50000), W.big_string("large", 100000)):
        wr.add_record(m.encode())
    log = bytes(dest)
    recs = W.wal_physical_records(log)
    offs = [o + 6 for o, _, _ in recs]
    lens = [ln + 1 for _, ln, _ in recs]
    got = gpu_batch(torch, dev, log, offs, lens, None, False)
    want = [W.unmask(W.decode_fixed_32(log[o:o + 4])) for o, _, _ in recs]
    assert list(got) == want
    scen = {s["name"]: s for s in wal_golden["scenarios"]}["fragmentation"]
    assert [u[1] for u in scen["crc_units"]] == want


def test_wal_writer_seeded_masked(torch_dev):
    """Batched form of log_writer.rs:123-125: mask(extend(type_crc[t], payload))."""
    torch, dev = torch_dev
    dest = bytearray()
    wr = W.Writer(dest)
    rnd = W.Random(301)
    for i in range(300):
        wr.add_record(W.random_skewed_string(i, rnd).encode())
    log = bytes(dest)
    recs = W.wal_physical_records(log)
    offs = [o + 7 for o, _, _ in recs]
    lens = [ln for _, ln, _ in recs]
    seeds = [wr.type_crc[t] for _, _, t in recs]
    got = gpu_batch(torch, dev, log, offs, lens, seeds, True)
    want = [W.decode_fixed_32(log[o:o + 4]) for o, _, _ in recs]
    assert list(got) == want


def test_host_api(kat, arena):
    c = np.array(kat["cases"], dtype=np.uint64)
    got = lvgpu.batch_host(arena, c[:, 0], c[:, 1], c[:, 2].astype(np.uint32), masked=True)
    assert np.array_equal(got, c[:, 4].astype(np.uint32))


def test_fill_matches_oracle_generator(torch_dev):
    torch, dev = torch_dev
    for begin, n in ((0, 4096), (13, 1001), (8, 64)):
        t = torch.empty(n, dtype=torch.uint8, device=dev)
        lvgpu.fill_splitmix(t, begin, 0x4C444231)
        torch.cuda.synchronize()
        h = ctypes.create_string_buffer(n)
        W.lib().oracle_fill_splitmix(h, begin, n, 0x4C444231)
        assert bytes(t.cpu().numpy()) == h.raw


def test_full_size_c3(torch_dev):
    """Config 3 at full size: 262,144 x 4 KiB = 1 GiB, bit-exact vs the oracle
    for every block, masked and unmasked, through both batch entry points."""
    torch, dev = torch_dev
    n, bl = 262144, 4096
    seed = 0x4C444231
    t = torch.empty(n * bl, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(t, 0, seed)
    offs = torch.arange(n, dtype=torch.int64, device=dev) * bl
    lens = torch.full((n,), bl, dtype=torch.int32, device=dev)
    out1 = lvgpu.batch(t, offs, lens)
    out2 = lvgpu.batch_strided(t, bl, bl, n, masked=True)
    torch.cuda.synchronize()
    host = t.cpu().numpy()
    want = oracle_batch(host.tobytes(), np.arange(n, dtype=np.uint64) * bl, np.full(n, bl, np.uint32), None, False)
    assert np.array_equal(out1.cpu().numpy().view(np.uint32), want)
    mk = np.array([W.mask(int(x)) for x in want[:4096]], dtype=np.uint32)
    got2 = out2.cpu().numpy().view(np.uint32)
    assert np.array_equal(got2[:4096], mk)
    # size-independent: unmask(masked) must reproduce every unmasked CRC
    assert np.array_equal(np.array([W.unmask(int(x)) for x in got2[-4096:]], dtype=np.uint32), want[-4096:])


def test_bad_arguments_raise(torch_dev):
    torch, dev = torch_dev
    with pytest.raises(lvgpu.LvError):
        lvgpu.lib()  # loads fine
        rc = lvgpu.lib().lv_crc32c_batch_device(None, None, None, None, None, 5, 0, None)
        lvgpu._check(rc)


@pytest.mark.parametrize("group", [None, 1, 4, 16, 64])
@pytest.mark.parametrize("block_len,stride_pad,n", [
    (64, 0, 1), (64, 16, 4097), (256, 0, 3001), (256, 48, 777), (1024, 0, 1025), (1024, 32, 64),
    (4096, 0, 262), (4096, 4096, 100), (8192, 16, 513), (65536, 0, 37), (1048576, 0, 3)])
@pytest.mark.parametrize("seeded", [False, True])
def test_uniform_block_kernel(torch_dev, group, block_len, stride_pad, n, seeded):
    """Aligned whole-batch blocks take the uniform-block kernel (SSTable
    blocks); ragged block counts leave partially filled waves."""
    torch, dev = torch_dev
    if group is not None and block_len % (64 * group):
        pytest.skip("block not a whole batch for this group size")
    stride = block_len + stride_pad
    rng = np.random.default_rng(block_len * 7 + n)
    total = stride * n
    t = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(t, 0, 0xB10C + n)
    seeds = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32) if seeded else None
    sd = None if seeds is None else torch.from_numpy(seeds.view(np.int32)).to(dev)
    out = lvgpu.batch_strided(t, stride, block_len, n, seed=sd, masked=seeded, group=group)
    torch.cuda.synchronize()
    host = t.cpu().numpy().tobytes()
    want = oracle_batch(host, np.arange(n, dtype=np.uint64) * stride, np.full(n, block_len, np.uint32), seeds, seeded)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)


def test_all_length_classes_one_batch(torch_dev):
    """One offsets-API call spanning every length class (<=256 B, <=2 KiB,
    <=32 KiB, >32 KiB up to 300 KiB), shuffled, misaligned, seeded: exercises
    the length sort and all four class launches together."""
    torch, dev = torch_dev
    rng = np.random.default_rng(44)
    lens = np.concatenate([rng.integers(0, 257, 3000), rng.integers(257, 2049, 1500),
                           rng.integers(2049, 32769, 600), rng.integers(32769, 300000, 40)]).astype(np.uint32)
    rng.shuffle(lens)
    gaps = rng.integers(0, 40, lens.size).astype(np.uint64)
    offs = np.zeros(lens.size, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1])
    total = int(offs[-1] + lens[-1]) + 16
    t = torch.empty(total, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(t, 0, 0x5EED)
    seeds = rng.integers(0, 2**32, lens.size, dtype=np.uint64).astype(np.uint32)
    host = t.cpu().numpy().tobytes()
    want = oracle_batch(host, offs, lens, seeds, True)
    o = torch.from_numpy(offs.astype(np.int64)).to(dev)
    ln = torch.from_numpy(lens.view(np.int32)).to(dev)
    sd = torch.from_numpy(seeds.view(np.int32)).to(dev)
    got = lvgpu.batch(t, o, ln, sd, masked=True).cpu().numpy().view(np.uint32)
    assert np.array_equal(got, want)
    # caller-owned workspace gives the same answer
    ws = torch.empty(lvgpu.workspace_bytes(lens.size), dtype=torch.uint8, device=dev)
    got2 = lvgpu.batch_ws(t, o, ln, ws, sd, masked=True).cpu().numpy().view(np.uint32)
    assert np.array_equal(got2, want)
    # single buffer, and two streams back to back (per-stream workspaces)
    one = lvgpu.batch(t, o[:1], ln[:1], sd[:1], masked=True).cpu().numpy().view(np.uint32)
    assert one[0] == want[0]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(s1):
        r1 = lvgpu.batch(t, o, ln, sd, masked=True, stream=s1)
    with torch.cuda.stream(s2):
        r2 = lvgpu.batch(t, torch.flip(o, [0]), torch.flip(ln, [0]), torch.flip(sd, [0]), masked=True,
                         stream=s2)
    torch.cuda.synchronize()
    assert np.array_equal(r1.cpu().numpy().view(np.uint32), want)
    assert np.array_equal(r2.cpu().numpy().view(np.uint32), want[::-1])


@pytest.mark.gpu
def test_batch_multi_devices(gpu):
    """lv_crc32c_batch_multi_devices: byte-balanced ranges over a device list
    (device 0 repeated on a 1-GPU box) equal the oracle; ngpu beyond the
    visible devices fails loudly."""
    import numpy as np
    import torch
    rng = np.random.default_rng(97)
    n = 5000
    lens = (32 * np.minimum(rng.zipf(1.1, size=n), 512)).astype(np.uint32)
    arena_n = int(lens.sum()) + 4096
    arena = rng.integers(0, 256, size=arena_n, dtype=np.uint8)
    offs = rng.integers(0, arena_n - lens.astype(np.int64), dtype=np.int64).astype(np.uint64)
    seeds = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    want = np.zeros(n, dtype=np.uint32)
    W.lib().oracle_batch(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, seeds.ctypes.data,
                         want.ctypes.data, n, 1)
    for devs in ([0], [0, 0], [0, 0, 0, 0, 0]):
        got = lvgpu.batch_multi(arena, offs, lens, seeds, masked=True, devices=devs)
        assert np.array_equal(got, want), devs
    assert np.array_equal(lvgpu.batch_multi(arena, offs, lens, seeds, masked=True, ngpu=1), want)
    with pytest.raises(lvgpu.LvError, match="device"):
        lvgpu.batch_multi(arena, offs, lens, seeds, ngpu=torch.cuda.device_count() + 1)


def test_batch_multi_ships_each_device_its_buffers(gpu):
    """A shuffled gather over a 96 MiB arena: every device range spans ~the
    whole arena, so the range's buffers are packed and each device receives
    its payload share plus metadata -- not the arena.
    Byte-packed buffers in index order ship their span as is.  CRCs equal
    the oracle either way."""
    import numpy as np
    rng = np.random.default_rng(123)
    n = 4000
    lens = rng.integers(0, 4000, size=n).astype(np.uint32)
    arena_n = 96 << 20
    arena = rng.integers(0, 256, size=arena_n, dtype=np.uint8)
    offs = rng.integers(0, arena_n - lens.astype(np.int64), dtype=np.int64).astype(np.uint64)
    payload = int(lens.sum(dtype=np.uint64))
    want = np.zeros(n, dtype=np.uint32)
    W.lib().oracle_batch(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, None, want.ctypes.data, n, 0)
    for devs in ([0], [0, 0, 0, 0]):
        before = lvgpu.device_counters(0)
        got = lvgpu.batch_multi(arena, offs, lens, None, devices=devs)
        moved = lvgpu.device_counters(0)["h2d"] - before["h2d"]
        assert np.array_equal(got, want), devs
        assert moved <= payload + 16 * n, (devs, moved, payload)
    # the page-locked pack buffer is cached per device: a repeat allocates nothing
    before = lvgpu.device_counters(0)
    got = lvgpu.batch_multi(arena, offs, lens, None, devices=[0, 0])
    assert np.array_equal(got, want)
    assert lvgpu.device_counters(0)["allocs"] == before["allocs"]
    # in index order and byte-packed: one span per range, no pack needed
    packed_offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    want2 = np.zeros(n, dtype=np.uint32)
    W.lib().oracle_batch(arena.ctypes.data, packed_offs.ctypes.data, lens.ctypes.data, None, want2.ctypes.data, n, 0)
    before = lvgpu.device_counters(0)
    got = lvgpu.batch_multi(arena, packed_offs, lens, None, devices=[0, 0, 0])
    moved = lvgpu.device_counters(0)["h2d"] - before["h2d"]
    assert np.array_equal(got, want2)
    assert moved <= payload + 16 * n


def test_batch_multi_packs_a_large_scatter_in_chunks(gpu):
    """A scattered gather whose range payload (~0.55 GiB, under 2/3 of its
    1 GiB span) exceeds the host pack chunk (256 MiB): the range ships in
    packed sub-ranges, a lone 260 MiB buffer straight from the arena; CRCs equal the oracle and the
    device still receives the payload, not the 1 GiB arena."""
    import numpy as np
    rng = np.random.default_rng(77)
    arena_n = 1 << 30
    arena = np.frombuffer(rng.bytes(arena_n), dtype=np.uint8)
    big = 260 << 20
    n_small = 150
    lens = np.full(n_small + 1, 2 << 20, dtype=np.uint32)
    lens[n_small // 2] = big
    lens[:n_small // 2] -= rng.integers(0, 4096, size=n_small // 2).astype(np.uint32)
    slots = rng.permutation((arena_n - big) // (2 << 20))[:n_small + 1].astype(np.uint64) * np.uint64(2 << 20)
    offs = slots.copy()
    offs[n_small // 2] = arena_n - big
    offs[0] = 0
    payload = int(lens.sum(dtype=np.uint64))
    want = np.zeros(lens.size, dtype=np.uint32)
    W.lib().oracle_batch(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, None, want.ctypes.data, lens.size, 0)
    before = lvgpu.device_counters(0)
    got = lvgpu.batch_multi(arena, offs, lens, None, devices=[0])
    moved = lvgpu.device_counters(0)["h2d"] - before["h2d"]
    assert np.array_equal(got, want)
    assert moved <= payload + 16 * lens.size + (4 << 20), (moved, payload)


def test_sorted_walk_edges(torch_dev, arena):
    """Offsets API edge geometry for the wave-uniform walk: lengths at the
    class edges (256/257, 2048/2049, 32768/32769) and at batch-count edges of
    each class (k*64, k*256, k*1024 +-1), every start alignment mod 16, seeded;
    empty buffers at the arena's first and last byte; one call holding them
    all shuffled, so waves mix batch counts that differ by one."""
    torch, dev = torch_dev
    rng = random.Random(2024)
    edges = {0, 1, 3, 4, 5, 15, 16, 17, 255, 256, 257, 2047, 2048, 2049, 32767, 32768, 32769, 65536}
    for unit in (64, 256, 1024):
        for k in range(1, 9):
            edges |= {k * unit - 1, k * unit, k * unit + 1}
    offs, lens = [], []
    for ln in sorted(edges):
        for mis in range(16):
            offs.append(4096 * rng.randrange(1, 150) + mis)
            lens.append(ln)
    offs += [0, len(arena), len(arena) - 1]
    lens += [0, 0, 1]
    order = list(range(len(offs)))
    rng.shuffle(order)
    offs = [offs[i] for i in order]
    lens = [lens[i] for i in order]
    seeds = [rng.getrandbits(32) for _ in offs]
    want = oracle_batch(arena, offs, lens, seeds, True)
    got = gpu_batch(torch, dev, arena, offs, lens, seeds, True)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(offs[i], lens[i]) for i in bad[:10]]


def test_aligned_row_geometry(torch_dev, arena):
    """The G = 16 classes walk rows on the absolute 256-B grid (merge_al):
    every start phase in the 256-B row (granule 0..15) x byte alignments, with
    lengths that put the last whole granule on every lane e = 0..15, plus
    single-batch, 32 KiB-edge and > 32 KiB buffers; seeded and masked."""
    torch, dev = torch_dev
    rng = random.Random(77)
    lengths = [2049 + 16 * t + rng.randrange(16) for t in range(16)] + [4096, 4097, 32768, 32769,
                                                                          40000 + rng.randrange(256)]
    offs, lens = [], []
    for ln in lengths:
        for ph in range(16):
            for mis in range(0, 16, 3):
                offs.append(256 * rng.randrange(1, 800) + 16 * ph + mis)
                lens.append(ln)
    seeds = [rng.getrandbits(32) for _ in offs]
    want = oracle_batch(arena, offs, lens, seeds, True)
    got = gpu_batch(torch, dev, arena, offs, lens, seeds, True)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(offs[i], lens[i]) for i in bad[:10]]


@pytest.mark.parametrize("workload", ["c2", "c4"])
def test_full_size_offsets_api(torch_dev, workload):
    """Configs 2 and 4 at full size (1,048,576 byte-packed buffers, 5.6-5.8 GiB,
    exactly bench.py's workloads): every CRC of lv_crc32c_batch_device
    bit-exact vs the oracle, unseeded, and seeded + masked with random seeds."""
    torch, dev = torch_dev
    import bench
    arena, off, ln, nbytes, _ = bench.build_workload(torch, lvgpu, workload, dev, 0)
    out = lvgpu.batch(arena, off, ln)
    rng = np.random.default_rng(11)
    seeds = rng.integers(0, 2**32, size=off.numel(), dtype=np.uint64).astype(np.uint32)
    sd = torch.from_numpy(seeds.view(np.int32)).to(dev)
    out_s = lvgpu.batch(arena, off, ln, sd, masked=True)
    torch.cuda.synchronize()
    host = arena.cpu().numpy()
    o = off.cpu().numpy().astype(np.uint64)
    n = ln.cpu().numpy().view(np.uint32)
    assert int(n.astype(np.uint64).sum()) == nbytes
    assert np.array_equal(out.cpu().numpy().view(np.uint32), oracle_batch(host, o, n, None, False))
    assert np.array_equal(out_s.cpu().numpy().view(np.uint32), oracle_batch(host, o, n, seeds, True))


def test_full_size_c5_shard(torch_dev):
    """Config 5's per-GPU shard at full size: 2,097,152 x 4 KiB = 8 GiB through
    the uniform-block kernel, every CRC bit-exact vs the oracle."""
    torch, dev = torch_dev
    import bench
    arena, off, ln, nbytes, _ = bench.build_workload(torch, lvgpu, "c5", dev, 0)
    n = off.numel()
    out = lvgpu.batch_strided(arena, 4096, 4096, n)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    host = arena.cpu().numpy()
    want = oracle_batch(host, np.arange(n, dtype=np.uint64) * 4096, np.full(n, 4096, np.uint32), None, False)
    assert np.array_equal(got, want)


def _oracle_uniform_range(byte_lo, n, bl, seed, chunk_blocks=16384, threads=16):
    """Oracle CRCs of n blocks of bl bytes whose bytes are the global splitmix
    arena from byte_lo on, generated on the host chunk by chunk (16 threads:
    the box's CPU share; ctypes drops the GIL inside the C calls)."""
    from concurrent.futures import ThreadPoolExecutor
    import threading
    L = W.lib()
    want = np.zeros(n, dtype=np.uint32)
    local = threading.local()
    offs = np.arange(chunk_blocks, dtype=np.uint64) * bl
    lens = np.full(chunk_blocks, bl, dtype=np.uint32)

    def one(c0):
        m = min(chunk_blocks, n - c0)
        buf = getattr(local, "buf", None)
        if buf is None:
            buf = local.buf = np.empty(chunk_blocks * bl, dtype=np.uint8)
        L.oracle_fill_splitmix(buf.ctypes.data, byte_lo + c0 * bl, m * bl, seed)
        L.oracle_batch(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data, None, want[c0:].ctypes.data, m, 0)
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(one, range(0, n, chunk_blocks)))
    return want


def test_full_size_c5_strong_world8(torch_dev):
    """BASELINE configs[4] at full size, as the driver's N = 8 line shards it:
    the global batch of 16,777,216 x 4 KiB = 64 GiB split by RankShard.uniform
    into 8 rank ranges, each generated at its byte_lo of the one global
    splitmix arena (bench.build_shard / c5_strong_record) and checksummed by
    the strided kernel, the ranges run one after another on this GPU.  Every
    one of the 16,777,216 CRCs equals the oracle's over host bytes generated
    at the same global offsets (so the ranges tile the arena where they
    belong, and no rank checksums another's bytes)."""
    torch, dev = torch_dev
    import bench
    from lvgpu.shard import RankShard
    world, bl = 8, 4096
    n_total = bench.C5_BLOCKS
    got_all = np.zeros(n_total, dtype=np.uint32)
    covered = 0
    for r in range(world):
        sh = RankShard.uniform(n_total, bl, r, world)
        assert sh.lo == covered and sh.byte_lo == sh.lo * bl
        arena = torch.empty(sh.byte_hi - sh.byte_lo, dtype=torch.uint8, device=dev)
        lvgpu.fill_splitmix(arena, sh.byte_lo, bench.PAYLOAD_SEED)
        out = lvgpu.batch_strided(arena, bl, bl, sh.n)
        torch.cuda.synchronize()
        got_all[sh.lo:sh.hi] = out.cpu().numpy().view(np.uint32)
        covered = sh.hi
        del arena, out
    assert covered == n_total
    want = _oracle_uniform_range(0, n_total, bl, bench.PAYLOAD_SEED)
    bad = np.nonzero(got_all != want)[0]
    assert bad.size == 0, f"{bad.size} CRCs differ, first blocks {bad[:8].tolist()}"


def test_many_buffers_chunked_sort(torch_dev):
    """n above one sort pass's 1024 x 4096 buffers (4,194,304): 5,000,000
    byte-packed buffers of 0-300 B (every small class, chunked length sort),
    seeded and masked, every CRC vs the oracle."""
    torch, dev = torch_dev
    rng = np.random.default_rng(5150)
    n = 5_000_000
    lens = rng.integers(0, 301, n).astype(np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    total = int(offs[-1] + lens[-1]) + 16
    t = torch.empty(total, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(t, 0, 0xB16)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    o = torch.from_numpy(offs.astype(np.int64)).to(dev)
    ln = torch.from_numpy(lens.view(np.int32)).to(dev)
    sd = torch.from_numpy(seeds.view(np.int32)).to(dev)
    got = lvgpu.batch(t, o, ln, sd, masked=True).cpu().numpy().view(np.uint32)
    want = oracle_batch(t.cpu().numpy(), offs, lens, seeds, True)
    assert np.array_equal(got, want)


def test_host_api_long_buffers(gpu):
    """lv_crc32c_batch_host cuts buffers over 1 MiB into 256 KiB pieces and
    joins them with GF(2) shifts: long buffers of whole and ragged piece
    counts, at odd offsets, beside short ones, seeded, masked and not."""
    rng = np.random.default_rng(1 << 20)
    arena = rng.integers(0, 256, size=24 << 20, dtype=np.uint8)
    lens = np.array([(1 << 20) + 1, 4 << 20, (5 << 20) + 12345, 3, 0, 4096, (1 << 20), 7777777],
                    dtype=np.uint32)
    offs = np.array([5, 3 << 20, 7, 11, 0, 99, (16 << 20) + 1, (24 << 20) - 7777777], dtype=np.uint64)
    seeds = rng.integers(0, 2**32, lens.size, dtype=np.uint64).astype(np.uint32)
    for masked in (False, True):
        want = oracle_batch(arena, offs, lens, seeds, masked)
        got = lvgpu.batch_host(arena, offs, lens, seeds, masked=masked)
        assert np.array_equal(got, want), masked
    want = oracle_batch(arena, offs, lens, None, False)
    assert np.array_equal(lvgpu.batch_host(arena, offs, lens, None), want)


@pytest.mark.parametrize("L,n", [(4096, 5000), (65536, 300), (1024, 70)])
def test_host_api_aligned_uniform_blocks(gpu, L, n):
    """lv_crc32c_batch_host passes its own LV_HINT_ALIGNED16 fact: uniform
    blocks at shuffled 16-B multiples run on the strided API's kernels
    (gathering their starts); one misaligned offset sends the same batch
    through the length sort.  Bit-exact vs the oracle both ways."""
    rng = np.random.default_rng(L + n)
    starts = np.cumsum(rng.integers(0, 3, n) * 16 + L) - L
    offs = rng.permutation(starts).astype(np.uint64)
    lens = np.full(n, L, dtype=np.uint32)
    arena = rng.integers(0, 256, size=int(starts[-1]) + L + 32, dtype=np.uint8)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    want = oracle_batch(arena, offs, lens, seeds, True)
    assert np.array_equal(lvgpu.batch_host(arena, offs, lens, seeds, masked=True), want)
    assert "gather" in lvgpu.last_kernel(), lvgpu.last_kernel()
    offs[n // 2] += 1
    want = oracle_batch(arena, offs, lens, seeds, True)
    assert np.array_equal(lvgpu.batch_host(arena, offs, lens, seeds, masked=True), want)
    assert "gather" not in lvgpu.last_kernel()


def test_two_threads_same_stream(torch_dev, arena):
    """Two host threads call the offsets API on the SAME stream (the default
    one) with different batch sizes: the library's per-stream sort workspace
    is locked from lookup through the last launch of a call, so neither
    call's sort passes interleave with the other's."""
    import threading
    torch, dev = torch_dev
    rng = np.random.default_rng(77)
    a = torch.frombuffer(bytearray(arena), dtype=torch.uint8).to(dev)
    cases = []
    for n in (5000, 23000):
        lens = rng.integers(0, 9000, size=n).astype(np.uint32)
        offs = rng.integers(0, len(arena) - 9000, size=n).astype(np.uint64)
        want = oracle_batch(arena, offs, lens, None, False)
        o = torch.from_numpy(offs.astype(np.int64)).to(dev)
        ln = torch.from_numpy(lens.view(np.int32)).to(dev)
        cases.append((o, ln, want))
    stream = torch.cuda.current_stream()
    errors = []

    def worker(k):
        o, ln, want = cases[k]
        try:
            for _ in range(30):
                out = lvgpu.batch(a, o, ln, stream=stream)
                torch.cuda.synchronize()
                got = out.cpu().numpy().view(np.uint32)
                if not np.array_equal(got, want):
                    errors.append(k)
                    return
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))
    th = [threading.Thread(target=worker, args=(k,)) for k in (0, 1)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert errors == []


def test_kernel_choice_query(torch_dev):
    """lv_crc32c_last_kernel names the path a call took: aligned whole-batch
    blocks run the uniform-block kernel (G by block count), unaligned strided
    geometry the generic strided kernel, the offsets API the fused small-batch
    kernel (<= 1,024 buffers) or the sort + class kernel."""
    torch, dev = torch_dev
    t = torch.zeros(4096 * 2048 + 64, dtype=torch.uint8, device=dev)
    lvgpu.batch_strided(t, 4096, 4096, 2048)
    assert lvgpu.last_kernel() == "crc32c_blocks_kernel<64>"  # few blocks: 64-lane groups
    lvgpu.batch_strided(t, 4096, 4096, 2048, group=16)
    assert lvgpu.last_kernel() == "crc32c_blocks_kernel<16>"
    lvgpu.batch_strided(t[1:], 4096, 4096, 2048)
    assert lvgpu.last_kernel().startswith("crc32c_batch_kernel<") and lvgpu.last_kernel().endswith(",strided>")
    o = torch.arange(16, dtype=torch.int64, device=dev) * 100
    ln = torch.full((16,), 100, dtype=torch.int32, device=dev)
    lvgpu.batch(t, o, ln)  # <= 1,024 buffers: split + walk in one launch, then the join
    assert lvgpu.last_kernel() == "crc32c_fused_small_kernel+combine_long_kernel"
    o = torch.arange(1025, dtype=torch.int64, device=dev) * 100
    ln = torch.full((1025,), 100, dtype=torch.int32, device=dev)
    lvgpu.batch(t, o, ln)
    assert lvgpu.last_kernel() == "sort+crc32c_classes_kernel+combine_long_kernel"
    torch.cuda.synchronize()


def _split_kernel(n, blen, cus):
    """The strided API's long-block split as lv_crc32c_batch_strided picks it
    (pick_split): 2^ps pieces of >= 4 KiB (whole KiB) until n 2^ps fills one
    pass of the grid; <= 16 pieces per block in one pass join in the same
    launch (FUSE), otherwise combine_pieces_kernel follows."""
    want, ps = 4 * cus * 16, 0
    while (n << ps) < want and ps < 12:
        s2 = 2 << ps
        if blen % s2 or (blen // s2) % 1024 or blen // s2 < 4096:
            break
        ps += 1
    if (1 << ps) <= 16 and (n << ps) <= 64 * cus:
        return "crc32c_blocks_kernel<16,pieces,fused>"
    if ps >= 11:
        return "crc32c_blocks_kernel<16,pieces>+combine_pieces_wg_kernel"
    return "crc32c_blocks_kernel<16,pieces>+combine_pieces_kernel"


@pytest.mark.parametrize("n,blen,seeded,masked", [(1, 16 << 20, False, False), (3, 1 << 20, True, True),
                                                  (64, 16 << 20, True, False), (1024, 65536, False, True),
                                                  (1024, 65536, True, False), (1001, 65536, True, True),
                                                  (2048, 32768, True, True), (4096, 16384, False, False),
                                                  (300, 65536, False, False), (1500, 65536, True, False),
                                                  (5, 8192, True, False), (200, 12288, False, False),
                                                  (7, 3 << 20, True, True), (2, 16 << 20, True, True),
                                                  (1, 8 << 20, False, True), (3, 12 << 20, True, False)])
def test_strided_long_block_split(torch_dev, n, blen, seeded, masked):
    """Few long blocks through lv_crc32c_batch_strided: each block is cut into
    2^k pieces that fill the grid and the piece registers are joined on the
    device (in the same launch for <= 16 pieces per block in one grid pass,
    else combine_pieces_kernel) -- the reference bench's 1 MiB and 16 MiB
    buffers (benches/crc32c.rs:59-60) and 1,024 x 64 KiB, bit-exact."""
    torch, dev = torch_dev
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    stride = blen + (0 if n % 2 else 4096)
    base = torch.empty(stride * n + 64, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(base, 0, 0x51D + n)
    rng = np.random.default_rng(n)
    seeds = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32) if seeded else None
    sd = None if seeds is None else torch.from_numpy(seeds.view(np.int32)).to(dev)
    out = lvgpu.batch_strided(base, stride, blen, n, seed=sd, masked=masked)
    assert lvgpu.last_kernel() == _split_kernel(n, blen, cus)
    got = out.cpu().numpy().view(np.uint32)
    host = base.cpu().numpy().tobytes()
    want = oracle_batch(host, np.arange(n, dtype=np.uint64) * stride, np.full(n, blen, np.uint32), seeds, masked)
    assert np.array_equal(got, want)


LONG_CASES = {
    "1MiB": [1 << 20],
    "16MiB": [16 << 20],
    "mixed": [16 << 20, 1 << 20, 37, 0, 70001, 5 << 20, 3, 16385, 40000],
    "1024x64KiB": [65536] * 1024,
    "300_ragged": [(1 << 20) + 13 * k for k in range(300)] + [100] * 50,
    "few_long_many_short": [9 << 20, 3 << 20] + [200 + k % 3000 for k in range(20000)],
    # the fused small-batch kernel (n <= 1,024, no sort) and the three-pass sort just past it
    "small_sort_2": [3 << 20, 17],
    "small_sort_1024": [(40000 + 977 * k) if k % 7 == 0 else (k * 37) % 3000 for k in range(1024)],
    "small_sort_1025": [(40000 + 977 * k) if k % 7 == 0 else (k * 37) % 3000 for k in range(1025)],
    # round 3: one-pass batches of the fused small-batch kernel -- 256-B-aligned
    # pieces take the one-round walk (all batches in flight), split buffers
    # whose pieces fall in one workgroup are joined there (mixed: some do, some
    # straddle two workgroups and go to combine_long_kernel)
    "1024x64KiB_aligned": [65536] * 1024,
    "16MiB_aligned": [16 << 20],
    "local_mixed": [65536, 1000] * 512,
    "local_mixed_aligned": [65536, 1000] * 512,
    "local_ragged_aligned": [40000 + 4096 * (k % 5) for k in range(700)],
}


@pytest.mark.parametrize("seeded", [True, False])
@pytest.mark.parametrize("case", sorted(LONG_CASES))
def test_offsets_api_long_buffers(torch_dev, case, seeded):
    """Long buffers through the device offsets API (the reference bench's 1 MiB
    and 16 MiB buffers, benches/crc32c.rs:59-60): the sort cuts buffers that
    are long relative to the batch into pieces after the sorted list, the
    class kernel walks them with the rest, and combine_long_kernel joins them.
    Alone, mixed with short ones, many at once, at odd start offsets, seeded
    or not, masked."""
    torch, dev = torch_dev
    sizes = LONG_CASES[case]
    aligned = case.endswith("_aligned")
    offs, pos = [], 0 if aligned else 3
    for sz in sizes:
        offs.append(pos)
        pos += sz + 5
        if aligned:
            pos = (pos + 255) & ~255
    arena = torch.empty(pos + 64, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(arena, 0, 0xB16 + len(sizes))
    rng = np.random.default_rng(len(sizes))
    seeds = rng.integers(0, 2**32, size=len(sizes), dtype=np.uint64).astype(np.uint32) if seeded else None
    o = torch.tensor(offs, dtype=torch.int64, device=dev)
    ln = torch.tensor(sizes, dtype=torch.int32, device=dev)
    sd = None if seeds is None else torch.from_numpy(seeds.view(np.int32)).to(dev)
    out = lvgpu.batch(arena, o, ln, sd, masked=True)
    got = out.cpu().numpy().view(np.uint32)
    want = oracle_batch(arena.cpu().numpy().tobytes(), offs, sizes, seeds, True)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(i), sizes[i]) for i in bad[:10]]


@pytest.mark.parametrize("n,size,seeded", [(20000, 3000, True), (5000, 200, False), (1, 100, True),
                                           (16384, 20000, True), (300, 20000, False), (70000, 4096, False),
                                           (40000, 2048, True)])
def test_offsets_api_one_key_batches(torch_dev, n, size, seeded):
    """Uniform lengths through the offsets API: when every buffer falls in one
    sort key and none can be split, sort_scatter is skipped and the class
    kernel reads off/len/seed in index order (kWsIdent); 300 x 20,000 B stays
    on the sorted path (class 2 above 16 KiB in a small batch: split into
    pieces).  Byte-packed offsets with gaps, seeded or not, masked."""
    torch, dev = torch_dev
    offs = 7 + np.arange(n, dtype=np.int64) * (size + 3)
    total = int(offs[-1]) + size + 64
    arena = torch.empty(total, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(arena, 0, 0x1DE + n)
    rng = np.random.default_rng(n)
    seeds = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32) if seeded else None
    o = torch.from_numpy(offs).to(dev)
    ln = torch.full((n,), size, dtype=torch.int32, device=dev)
    sd = None if seeds is None else torch.from_numpy(seeds.view(np.int32)).to(dev)
    out = lvgpu.batch(arena, o, ln, sd, masked=True)
    got = out.cpu().numpy().view(np.uint32)
    want = oracle_batch(arena.cpu().numpy().tobytes(), offs, np.full(n, size), seeds, True)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, bad[:10]


@pytest.mark.parametrize("trial", range(6))
def test_offsets_api_small_batches_random(torch_dev, trial):
    """Random batches of 1-1,024 buffers (the fused small-batch kernel, no sort):
    lengths 0 to 3 MiB with a few long ones split into pieces, overlapping
    and unaligned offsets, seeded or not, masked or not -- every CRC against
    the oracle."""
    torch, dev = torch_dev
    rng = np.random.default_rng(1000 + trial)
    n = int(rng.integers(1, 1025))
    lens = rng.integers(0, 5000, size=n)
    longs = rng.random(n) < 0.02
    lens[longs] = rng.integers(16385, 3 << 20, size=int(longs.sum()))
    total = int(lens.max()) + 4 * n + 4096
    arena = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(arena, 0, 0x5A11 + trial)
    offs = np.array([int(rng.integers(0, total - int(l) + 1)) for l in lens], dtype=np.int64)
    seeded, masked = trial % 2 == 0, trial % 3 == 0
    seeds = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32) if seeded else None
    o = torch.from_numpy(offs).to(dev)
    ln = torch.from_numpy(lens.astype(np.int32)).to(dev)
    sd = None if seeds is None else torch.from_numpy(seeds.view(np.int32)).to(dev)
    out = lvgpu.batch(arena, o, ln, sd, masked=masked)
    got = out.cpu().numpy().view(np.uint32)
    want = oracle_batch(arena.cpu().numpy().tobytes(), offs, lens, seeds, masked)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(i), int(lens[i])) for i in bad[:10]]


@pytest.mark.parametrize("trial", range(8))
def test_offsets_api_one_pass_local_joins_random(torch_dev, trial):
    """Random one-pass batches of the fused small-batch kernel built so that
    split buffers of 3-64 pieces mix with short ones: some buffers' pieces
    fall in one workgroup's units (joined in the kernel), some straddle two
    (combine_long_kernel), at 256-B-aligned or odd offsets, seeded or not,
    masked or not -- every CRC against the oracle."""
    torch, dev = torch_dev
    rng = np.random.default_rng(2000 + trial)
    n = int(rng.integers(2, 1025))
    lens = rng.integers(0, 4000, size=n)
    split = rng.random(n) < 0.3
    lens[split] = rng.integers(16385, 64 * 4096, size=int(split.sum()))  # 4 KiB pieces: 5-64 each
    aligned = trial % 2 == 0
    offs, pos = [], 0
    for sz in lens:
        offs.append(pos)
        pos += int(sz) + int(rng.integers(0, 9))
        if aligned:
            pos = (pos + 255) & ~255
    arena = torch.empty(pos + 64, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(arena, 0, 0x10CA1 + trial)
    seeded, masked = trial % 4 < 2, trial % 3 == 0
    seeds = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32) if seeded else None
    o = torch.tensor(offs, dtype=torch.int64, device=dev)
    ln = torch.from_numpy(lens.astype(np.int32)).to(dev)
    sd = None if seeds is None else torch.from_numpy(seeds.view(np.int32)).to(dev)
    out = lvgpu.batch(arena, o, ln, sd, masked=masked)
    assert lvgpu.last_kernel() == "crc32c_fused_small_kernel+combine_long_kernel"
    got = out.cpu().numpy().view(np.uint32)
    want = oracle_batch(arena.cpu().numpy().tobytes(), np.array(offs, dtype=np.int64), lens, seeds, masked)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(i), int(lens[i])) for i in bad[:10]]


# Split buffers of the fused small-batch kernel that straddle workgroups
# (joined by combine_long_kernel): one-pass batches (static per-workgroup
# rounds) and the round-robin pool (> 16,384 units)
STRADDLE_CASES = {
    "static_16x1MiB": [1 << 20] * 16,  # 256 pieces each over 16 workgroups
    "static_16MiB": [16 << 20],  # 4,096 pieces over every workgroup
    "static_mixed": [3 << 20, 70000, 17, 0, 5 << 20] + [300] * 200,
    "pool_1000x65KiB": [66560] * 1000,  # 17 pieces each: 17,000 units
    "pool_big_and_small": [32 << 20] + [98305] * 1023,  # 4,096 + 1,023 x 13 pieces
}


@pytest.mark.parametrize("api", ["library_ws", "caller_ws"])
@pytest.mark.parametrize("case", sorted(STRADDLE_CASES))
def test_offsets_api_straddling_joins_repeat(torch_dev, case, api):
    """Split buffers whose pieces straddle workgroups of the fused small-batch
    kernel, joined by combine_long_kernel from the long records the fused
    kernel wrote.  Three calls in a row on one stream -- seeded, unseeded
    masked, seeded again, with a sorted-path call (n > 1,024) on the same
    workspace in between -- through the library's workspace and a dirty
    caller workspace, every CRC against the oracle each time (no state may
    leak from one call into the next)."""
    torch, dev = torch_dev
    sizes = STRADDLE_CASES[case]
    offs, pos = [], 3
    for sz in sizes:
        offs.append(pos)
        pos += sz + 5
    arena = torch.empty(pos + 64, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(arena, 0, 0xC0DE + len(sizes))
    host = arena.cpu().numpy().tobytes()
    rng = np.random.default_rng(len(sizes))
    seeds = rng.integers(0, 2**32, size=len(sizes), dtype=np.uint64).astype(np.uint32)
    o = torch.tensor(offs, dtype=torch.int64, device=dev)
    ln = torch.tensor(sizes, dtype=torch.int32, device=dev)
    sd = torch.from_numpy(seeds.view(np.int32)).to(dev)
    want_s = oracle_batch(host, offs, sizes, seeds, False)
    want_m = oracle_batch(host, offs, sizes, None, True)
    ws = None
    if api == "caller_ws":  # a dirty workspace
        nb = max(lvgpu.workspace_bytes(len(sizes)), lvgpu.workspace_bytes(1100))
        ws = torch.full((nb,), 0xff, dtype=torch.uint8, device=dev)

    def run(seed, masked):
        if ws is None:
            out = lvgpu.batch(arena, o, ln, seed, masked=masked)
        else:
            out = lvgpu.batch_ws(arena, o, ln, ws, seed, masked=masked)
        assert lvgpu.last_kernel() == "crc32c_fused_small_kernel+combine_long_kernel"
        return out.cpu().numpy().view(np.uint32)

    for k, (seed, masked, want) in enumerate([(sd, False, want_s), (None, True, want_m), (sd, False, want_s)]):
        got = run(seed, masked)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (k, [(int(i), sizes[i]) for i in bad[:10]])
        if k == 0:  # the sorted path on the same stream / workspace in between
            o2 = torch.arange(1100, dtype=torch.int64, device=dev) * 50
            l2 = torch.full((1100,), 40000, dtype=torch.int32, device=dev)
            a2 = torch.empty(1100 * 50 + 40064, dtype=torch.uint8, device=dev)
            lvgpu.fill_splitmix(a2, 0, 7)
            if ws is None:
                lvgpu.batch(a2, o2, l2)
            else:
                lvgpu.batch_ws(a2, o2, l2, ws)
            assert lvgpu.last_kernel() == "sort+crc32c_classes_kernel+combine_long_kernel"


@pytest.mark.parametrize("n,L,distinct", [(300, 1 << 30, 5), (2000, 256 << 20, 7), (40000, (8 << 20) + 1, 3)])
def test_offsets_api_huge_batch_piece_budget(torch_dev, n, L, distinct):
    """Batches of 300-500 GiB of heavily overlapping buffers: the
    piece length P must stay >= batch bytes / 16,384 however large the batch,
    or the split overruns the piece budget (300 x 1 GiB: 256 pieces each,
    76,800 > 65,536) or the long-record budget (40,000 x 8 MiB: 32,768
    records).  The buffers repeat `distinct` (offset, length) pairs, so the
    oracle runs once per pair; every output is checked."""
    torch, dev = torch_dev
    arena = torch.empty(L + 4096, dtype=torch.uint8, device=dev)
    lvgpu.fill_splitmix(arena, 0, 0xB16B + n)
    k = np.arange(n) % distinct
    offs = (k * 517 + 3).astype(np.int64)
    lens = (L - k * 1031).astype(np.int64)
    assert int((offs + lens).max()) <= arena.numel()
    o = torch.from_numpy(offs).to(dev)
    ln = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev)
    out = lvgpu.batch(arena, o, ln, None, masked=True)
    got = out.cpu().numpy().view(np.uint32)
    host = arena.cpu().numpy().tobytes()
    want_pair = oracle_batch(host, offs[:distinct], lens[:distinct], None, True)
    want = want_pair[k]
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad.size, bad[:10])


HINT_CASES = {
    # name: (lengths, offsets layout, join expected with the hint)
    "uniform_1024x64KiB": (lambda r: np.full(1024, 65536), "packed", False),  # every split buffer is local
    "uniform_1x16MiB": (lambda r: np.full(1, 16 << 20), "packed", True),      # 4,096 pieces straddle
    "uniform_16x1MiB": (lambda r: np.full(16, 1 << 20), "odd", True),
    "uniform_300x4KiB": (lambda r: np.full(300, 4096), "odd", False),          # nothing splits
    "small_mixed_fused": (lambda r: r.integers(0, 16385, 900), "odd", False),  # <= 16 KiB never splits
    "sorted_no_split": (lambda r: r.integers(0, 9000, 5000), "odd", True),     # the sort; its join launch unsorts
    "sorted_long": (lambda r: np.concatenate([r.integers(0, 5000, 3000), [3 << 20, 70000]]), "odd", True),
    "fused_long_ragged": (lambda r: np.concatenate([r.integers(0, 300, 100), [1 << 20, 5 << 20]]), "odd", True),
    # uniform, > 1,024 buffers, nothing splits: the class kernel alone, no sort (class 0 .. 3)
    "uniform_5000x100B": (lambda r: np.full(5000, 100), "odd", False),
    "uniform_3000x1500B": (lambda r: np.full(3000, 1500), "packed", False),
    "uniform_2000x16KiB": (lambda r: np.full(2000, 16384), "odd", False),
    "uniform_8200x40000B": (lambda r: np.full(8200, 40000), "overlap", False),  # class 3, 8,200 > 2 x 40000 / 16384
    "uniform_1025x0B": (lambda r: np.zeros(1025), "packed", False),
    # uniform, > 1,024 buffers, split: the sort path and the join
    "uniform_1100x160KiB": (lambda r: np.full(1100, 160 << 10), "overlap", True),
}


def _hint_kernel(n, hint, join):
    """The launch lv_crc32c_batch_device_hint picks (classes.hip)."""
    if n <= 1024:
        return "crc32c_fused_small_kernel" + ("+combine_long_kernel" if join else "")
    if hint.uniform and not join:
        return "hint_len_kernel+crc32c_classes_kernel"  # a host-known identity list: no sort (lengths checked)
    return "sort+crc32c_classes_kernel" + ("+combine_long_kernel" if join else "")


@pytest.mark.parametrize("case", sorted(HINT_CASES))
@pytest.mark.parametrize("seeded", [False, True])
def test_offsets_api_with_hint(torch_dev, case, seeded):
    """lv_crc32c_batch_device_hint: exact host-side
    facts (total bytes, max length, uniform) let the library leave out the
    long-buffer join when no buffer can split, or when every split buffer of
    a uniform small batch is joined inside the walk; CRCs bit-exact vs the
    oracle with and without the hint, and the join launched exactly when a
    split buffer straddles workgroups."""
    torch, dev = torch_dev
    rng = np.random.default_rng(sum(map(ord, case)) * 7919)
    make, layout, join = HINT_CASES[case]
    lens = np.asarray(make(rng), dtype=np.uint32)
    n = lens.size
    if layout == "overlap":  # every buffer inside one window (keeps big batches' arenas small)
        offs = rng.integers(0, 4096, n).astype(np.uint64)
        pos = int(lens.max()) + 4096
    else:
        gaps = rng.integers(0, 16, n) if layout == "odd" else np.zeros(n, dtype=np.int64)
        offs = np.zeros(n, dtype=np.uint64)
        pos = 0
        for i in range(n):
            pos += int(gaps[i])
            offs[i] = pos
            pos += int(lens[i])
    arena = rng.integers(0, 256, pos + 16, dtype=np.uint8).tobytes()
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) if seeded else None
    want = oracle_batch(arena, offs, lens, seeds, True)
    a = torch.frombuffer(bytearray(arena), dtype=torch.uint8).to(dev)
    o = torch.from_numpy(offs.astype(np.int64)).to(dev)
    ln = torch.from_numpy(lens.view(np.int32)).to(dev)
    sd = None if seeds is None else torch.from_numpy(seeds.view(np.int32)).to(dev)
    hint = lvgpu.hint_for(lens)
    assert bool(hint.uniform) == case.startswith("uniform")
    out = lvgpu.batch_hint(a, o, ln, hint, seed=sd, masked=True)
    kern = lvgpu.last_kernel()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
    assert kern == _hint_kernel(n, hint, join), kern
    # the same call without the hint, and with a caller workspace
    ws = torch.empty(lvgpu.workspace_bytes(n), dtype=torch.uint8, device=dev)
    out2 = lvgpu.batch_hint(a, o, ln, None, seed=sd, masked=True, workspace=ws)
    assert "combine_long_kernel" in lvgpu.last_kernel()
    out3 = lvgpu.batch_hint(a, o, ln, hint, seed=sd, masked=True, workspace=ws)
    torch.cuda.synchronize()
    assert np.array_equal(out2.cpu().numpy().view(np.uint32), want)
    assert np.array_equal(out3.cpu().numpy().view(np.uint32), want)


ALIGNED_HINT_CASES = {
    # name: (n, length, kernel substring with LV_HINT_ALIGNED16)
    "20000x4KiB": (20000, 4096, "crc32c_blocks_kernel<16,gather>"),
    "3000x1KiB": (3000, 1024, "crc32c_blocks_kernel<16,gather>"),
    "40x4KiB_g64": (40, 4096, "crc32c_blocks_kernel<64,gather>"),
    "1024x64KiB": (1024, 65536, "crc32c_blocks_kernel<16,pieces,fused,gather>"),
    "2000x8KiB": (2000, 8192, "crc32c_blocks_kernel<16,pieces,fused,gather>"),
    "16x1MiB": (16, 1 << 20, "crc32c_blocks_kernel<16,pieces,gather>+combine_pieces_kernel"),
    "1x16MiB": (1, 16 << 20, "crc32c_blocks_kernel<16,pieces,gather>+combine_pieces_wg_kernel"),
    "5000x4000B": (5000, 4000, "hint_len_kernel+crc32c_classes_kernel"),  # not whole 1 KiB batches: the identity list
    "600x1000B": (600, 1000, "crc32c_fused_small_kernel"),
}


@pytest.mark.parametrize("case", sorted(ALIGNED_HINT_CASES))
@pytest.mark.parametrize("seeded", [False, True])
def test_offsets_api_with_aligned_hint(torch_dev, case, seeded):
    """LV_HINT_ALIGNED16: a uniform batch of 16-B aligned buffers whose
    length is whole 1 KiB batches runs on the strided API's kernels
    (crc32c_blocks_kernel, its long-block split and joins) with each buffer's
    start read from d_off.  Offsets are shuffled with gaps, so the walk must
    gather; CRCs bit-exact vs the oracle with the library's and a caller's
    workspace, the join query agrees with the launch, and a misaligned arena
    ignores the bit."""
    torch, dev = torch_dev
    n, L, kern = ALIGNED_HINT_CASES[case]
    rng = np.random.default_rng(sum(map(ord, case)) * 104729 + seeded)
    gaps = rng.integers(0, 4, n) * 16
    Lp = -(-L // 16) * 16
    starts = np.cumsum(gaps + Lp) - Lp  # aligned, in arena order
    offs = rng.permutation(starts).astype(np.uint64)
    lens = np.full(n, L, dtype=np.uint32)
    size = int(starts[-1]) + L + 64
    arena = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) if seeded else None
    want = oracle_batch(arena, offs, lens, seeds, True)
    a = torch.frombuffer(bytearray(arena), dtype=torch.uint8).to(dev)
    o = torch.from_numpy(offs.astype(np.int64)).to(dev)
    ln = torch.from_numpy(lens.view(np.int32)).to(dev)
    sd = None if seeds is None else torch.from_numpy(seeds.view(np.int32)).to(dev)
    hint = lvgpu.hint_for(lens, offs)
    assert hint.uniform == lvgpu.HINT_UNIFORM | lvgpu.HINT_ALIGNED16
    out = lvgpu.batch_hint(a, o, ln, hint, seed=sd, masked=True)
    k1 = lvgpu.last_kernel()
    ws = torch.empty(lvgpu.workspace_bytes(n), dtype=torch.uint8, device=dev)
    out2 = lvgpu.batch_hint(a, o, ln, hint, seed=sd, masked=True, workspace=ws)
    k2 = lvgpu.last_kernel()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
    assert np.array_equal(out2.cpu().numpy().view(np.uint32), want)
    assert k1 == k2 and k1.startswith(kern), k1
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    joined = "combine" in k1
    assert lvgpu.lib().lv_crc32c_hint_needs_join(ctypes.addressof(hint), n, cus) == int(joined)
    # the same offsets against an arena 8 bytes off 16-B alignment: the bit is ignored
    a8 = torch.empty(size + 8, dtype=torch.uint8, device=dev)[8:]
    a8.copy_(a)
    out3 = lvgpu.batch_hint(a8, o, ln, hint, seed=sd, masked=True)
    k3 = lvgpu.last_kernel()
    torch.cuda.synchronize()
    assert np.array_equal(out3.cpu().numpy().view(np.uint32), want)
    assert "gather" not in k3, k3


def test_hint_rejects_inconsistent_uniform(torch_dev):
    torch, dev = torch_dev
    a = torch.zeros(64, dtype=torch.uint8, device=dev)
    o = torch.zeros(2, dtype=torch.int64, device=dev)
    ln = torch.full((2,), 8, dtype=torch.int32, device=dev)
    with pytest.raises(lvgpu.LvError):
        lvgpu.batch_hint(a, o, ln, lvgpu.BatchHint(17, 8, 1))


def test_hint_rejects_unknown_uniform_bits(torch_dev):
    """`uniform` is 0, LV_HINT_UNIFORM or LV_HINT_UNIFORM |
    LV_HINT_ALIGNED16; ALIGNED16 alone or unknown bits are LV_ERR_INVALID."""
    torch, dev = torch_dev
    a = torch.zeros(64, dtype=torch.uint8, device=dev)
    o = torch.zeros(2, dtype=torch.int64, device=dev)
    ln = torch.full((2,), 16, dtype=torch.int32, device=dev)
    for bad in (lvgpu.HINT_ALIGNED16, 4, 5, 0x80000001):
        with pytest.raises(lvgpu.LvError):
            lvgpu.batch_hint(a, o, ln, lvgpu.BatchHint(32, 16, bad))


def _hint_case(torch, dev, rng, n, L, aligned, seeded=False, slack=1 << 16):
    """n buffers of L bytes at (16-B aligned if `aligned`) shuffled offsets in
    an arena with `slack` bytes after the last one."""
    Lp = -(-L // 16) * 16 + (0 if aligned else 3)
    starts = np.arange(n, dtype=np.uint64) * Lp
    offs = rng.permutation(starts).astype(np.uint64)
    arena = rng.integers(0, 256, int(starts[-1]) + L + slack, dtype=np.uint8).tobytes()
    a = torch.frombuffer(bytearray(arena), dtype=torch.uint8).to(dev)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) if seeded else None
    sd = None if seeds is None else torch.from_numpy(seeds.view(np.int32)).to(dev)
    return arena, a, offs, seeds, sd


# name: (n, L, aligned hint, how the device arrays contradict the hint, bits, kernel)
HINT_LIE_CASES = {
    # (the blocks kernel's group size is the strided plan's, G = 16 or 64 by CU count)
    "gather_misaligned_offset": (3000, 4096, True, "misalign", lvgpu.HINT_ERR_MISALIGNED, "crc32c_blocks_kernel<"),
    "gather_understated_max_len": (3000, 4096, True, "longer", lvgpu.HINT_ERR_NOT_UNIFORM, "crc32c_blocks_kernel<"),
    "gather_pieces_misaligned": (1024, 65536, True, "misalign", lvgpu.HINT_ERR_MISALIGNED,
                                 "crc32c_blocks_kernel<16,pieces,fused,gather>"),
    "gather_pieces_shorter": (16, 1 << 20, True, "shorter", lvgpu.HINT_ERR_NOT_UNIFORM,
                              "crc32c_blocks_kernel<16,pieces,gather>+combine_pieces_kernel"),
    "identity_understated": (5000, 4000, False, "longer", lvgpu.HINT_ERR_NOT_UNIFORM,
                             "hint_len_kernel+crc32c_classes_kernel"),
    # (the fused kernel sums every length too: a shorter one also misses the total)
    "fused_uniform_shorter": (600, 1000, False, "shorter", lvgpu.HINT_ERR_NOT_UNIFORM | lvgpu.HINT_ERR_TOTAL,
                              "crc32c_fused_small_kernel"),
    "fused_understated_max": (600, 1000, False, "nonuniform_longer",
                              lvgpu.HINT_ERR_LONGER | lvgpu.HINT_ERR_TOTAL, "crc32c_fused_small_kernel"),
}


@pytest.mark.parametrize("case", sorted(HINT_LIE_CASES))
def test_wrong_hint_is_reported(torch_dev, case):
    """a hint the device arrays contradict is reported by
    lv_crc32c_batch_check (LV_ERR_HINT with the violated facts), not answered
    with silently wrong CRCs; the same arrays with an exact hint check clean,
    and the record clears after a check."""
    torch, dev = torch_dev
    n, L, aligned, lie, bits, kern = HINT_LIE_CASES[case]
    rng = np.random.default_rng(sum(map(ord, case)))
    arena, a, offs, seeds, sd = _hint_case(torch, dev, rng, n, L, aligned)
    lens = np.full(n, L, dtype=np.uint32)
    hint = lvgpu.hint_for(lens, offs if aligned else None)
    assert hint.uniform == (3 if aligned else 1)
    lvgpu.batch_check()  # nothing recorded on this stream yet (or cleared)
    # the exact hint: CRCs right, no violation
    o = torch.from_numpy(offs.astype(np.int64)).to(dev)
    ln = torch.from_numpy(lens.view(np.int32)).to(dev)
    out = lvgpu.batch_hint(a, o, ln, hint, masked=True)
    assert lvgpu.last_kernel().startswith(kern), lvgpu.last_kernel()
    assert ("gather" in lvgpu.last_kernel()) == aligned, lvgpu.last_kernel()
    lvgpu.batch_check()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), oracle_batch(arena, offs, lens, None, True))
    # now the device arrays contradict the (unchanged) hint
    k = int(rng.integers(0, n))
    offs2, lens2 = offs.copy(), lens.copy()
    if lie == "misalign":
        offs2[k] += 8
    elif lie == "longer":
        lens2[k] = L + 5
    elif lie == "shorter":
        lens2[k] = L - 16
    elif lie == "nonuniform_longer":  # a non-uniform hint whose max_len is understated
        lens2[: n // 2] = L // 2
        hint = lvgpu.hint_for(lens2)
        lens2[k] = L + 1
    o2 = torch.from_numpy(offs2.astype(np.int64)).to(dev)
    ln2 = torch.from_numpy(lens2.view(np.int32)).to(dev)
    lvgpu.batch_hint(a, o2, ln2, hint, masked=True)
    with pytest.raises(lvgpu.HintViolation) as ei:
        lvgpu.batch_check()
    assert ei.value.violations == bits, (hex(ei.value.violations), lvgpu.last_kernel())
    lvgpu.batch_check()  # the record was cleared
    # a caller workspace takes the same checks
    ws = torch.empty(lvgpu.workspace_bytes(n), dtype=torch.uint8, device=dev)
    lvgpu.batch_hint(a, o2, ln2, hint, masked=True, workspace=ws)
    with pytest.raises(lvgpu.HintViolation):
        lvgpu.batch_check()


@pytest.mark.parametrize("n,L", [(64, 17 << 10), (200, 20 << 10), (1024, 64 << 10)])
def test_aligned_hint_on_misaligned_arena_joins(torch_dev, n, L):
    """with LV_HINT_ALIGNED16 but an arena pointer off
    16-B alignment the library ignores the bit -- and its join decision must
    not assume the aligned path ran.  64 x 17 KiB and 200 x 20 KiB split into
    pieces that straddle workgroups on any CU count, so the fused walk needs
    combine_long_kernel; CRCs bit-exact vs the oracle."""
    torch, dev = torch_dev
    rng = np.random.default_rng(n * 31 + L)
    arena, a, offs, _, _ = _hint_case(torch, dev, rng, n, L, True, slack=64)
    lens = np.full(n, L, dtype=np.uint32)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    hint = lvgpu.hint_for(lens, offs)
    assert hint.uniform == 3
    a8 = torch.empty(a.numel() + 8, dtype=torch.uint8, device=dev)[8:]
    a8.copy_(a)
    o = torch.from_numpy(offs.astype(np.int64)).to(dev)
    ln = torch.from_numpy(lens.view(np.int32)).to(dev)
    sd = torch.from_numpy(seeds.view(np.int32)).to(dev)
    out = lvgpu.batch_hint(a8, o, ln, hint, seed=sd, masked=True)
    kern = lvgpu.last_kernel()
    lvgpu.batch_check()
    assert "gather" not in kern, kern
    if (n, L) != (1024, 64 << 10):
        assert "combine_long_kernel" in kern, kern
    assert np.array_equal(out.cpu().numpy().view(np.uint32), oracle_batch(arena, offs, lens, seeds, True))
