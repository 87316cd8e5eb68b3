"""table/format.rs codecs and SSTable block trailers.

CPU: the oracle (oracle/table_oracle.py) against the reference's own format
and varint tests (format.rs:107-147, coding.rs:481-510) and the committed
fixture; the product's codecs (lv_sst_block_handle_*/lv_sst_footer_*)
against the same fixture and the reference error strings.
GPU: lv_sst_seal_blocks_device / lv_sst_verify_blocks_* against the oracle
trailer; the trailer layout itself is parity-unpinned (table.h)."""
import json
import os

import numpy as np
import pytest

import table_oracle as T
import wal_oracle as W
from conftest import GOLDEN


@pytest.fixture(scope="module")
def tfix():
    with open(os.path.join(GOLDEN, "table_format.json")) as f:
        return json.load(f)


def test_oracle_reference_format_tests():
    b = bytearray()
    T.BlockHandle(10, 20).encode_to(b)                                    # format.rs:107-123
    assert T.BlockHandle.decode_from(bytes(b)) == (T.BlockHandle(10, 20), len(b))
    f = bytearray()
    ft = T.Footer(T.BlockHandle(50, 100), T.BlockHandle(200, 400))        # format.rs:125-147
    ft.encode_to(f)
    assert len(f) == T.FOOTER_ENCODED_LENGTH
    assert T.Footer.decode_from(bytes(f)) == ft
    v = T.encode_varint_64(1 << 60)                                       # coding.rs:502-510
    assert T.decode_varint_64(v + bytes(10 - len(v))) == (1 << 60, len(v))
    r = W.Random(0xBAAAAAAD)                                              # coding.rs:481-489
    for _ in range(1000):
        x = r.next()
        assert T.varint_length(x) == len(T.encode_varint_64(x))


def test_oracle_matches_fixture(tfix, arena):
    for h in tfix["block_handles"]:
        b = bytearray()
        T.BlockHandle(h["offset"], h["size"]).encode_to(b)
        assert b.hex() == h["hex"]
    for f in tfix["footers"]:
        b = bytearray()
        T.Footer(T.BlockHandle(*f["metaindex"]), T.BlockHandle(*f["index"])).encode_to(b)
        assert b.hex() == f["hex"]
    for v, hx in tfix["varints"]:
        assert T.encode_varint_64(v).hex() == hx
    for off, ln, ctype, hx in tfix["trailers"]:
        assert T.block_trailer(arena[off:off + ln], ctype).hex() == hx


def test_product_codecs_match_fixture(tfix):
    from lvgpu import table as LT
    for h in tfix["block_handles"]:
        b = bytearray()
        LT.BlockHandle(h["offset"], h["size"]).encode_to(b)
        assert b.hex() == h["hex"]
        raw = bytes.fromhex(h["hex"])
        assert LT.BlockHandle.decode_from(raw + b"\xff\x01") == (LT.BlockHandle(h["offset"], h["size"]), len(raw))
    for f in tfix["footers"]:
        ft = LT.Footer(LT.BlockHandle(*f["metaindex"]), LT.BlockHandle(*f["index"]))
        assert ft.encode().hex() == f["hex"]
        assert LT.Footer.decode_from(bytes.fromhex(f["hex"])) == ft


def test_product_codec_errors():
    from lvgpu import LvError, table as LT
    with pytest.raises(LT.Corruption, match="bad handle"):
        LT.BlockHandle.decode_from(b"\x80\x80")            # unterminated varint
    with pytest.raises(LT.Corruption, match="bad handle"):
        LT.BlockHandle.decode_from(b"\x05")                # offset only
    with pytest.raises(LT.Corruption, match="bad handle"):
        LT.BlockHandle.decode_from(b"\xff" * 11 + b"\x01")  # > 10 varint bytes
    good = LT.Footer(LT.BlockHandle(1, 2), LT.BlockHandle(3, 4)).encode()
    with pytest.raises(LT.Corruption, match="not a sstable"):
        LT.Footer.decode_from(good[:-1] + b"\x00")
    with pytest.raises(LvError):
        LT.Footer.decode_from(good[:47])
    # oracle agrees on the same malformed inputs
    for bad in (b"\x80\x80", b"\x05", b"\xff" * 11 + b"\x01"):
        with pytest.raises(T.Corruption):
            T.BlockHandle.decode_from(bad)
    with pytest.raises(T.Corruption):
        T.Footer.decode_from(good[:-1] + b"\x00")


def _make_table(rng, nblocks, sizes=None):
    """Synthetic table: blocks with 5-byte trailers (left zero), then a footer."""
    handles, parts, pos = [], [], 0
    for k in range(nblocks):
        sz = int(sizes[k]) if sizes is not None else int(rng.choice([0, 1, 4096, int(rng.integers(0, 70000))]))
        parts.append(rng.integers(0, 256, size=sz, dtype=np.uint8).tobytes() + bytes(T.BLOCK_TRAILER_SIZE))
        handles.append((pos, sz))
        pos += sz + T.BLOCK_TRAILER_SIZE
    return bytearray(b"".join(parts)), handles


def _oracle_seal(file, handles, types):
    f = bytearray(file)
    for (o, sz), t in zip(handles, types):
        f[o + sz:o + sz + 5] = T.block_trailer(bytes(f[o:o + sz]), t)
    return bytes(f)


@pytest.mark.gpu
def test_gpu_seal_and_verify(gpu):
    import torch
    from lvgpu import table as LT
    rng = np.random.default_rng(71)
    file, handles = _make_table(rng, 300)
    types = rng.integers(0, 2, size=len(handles)).astype(np.uint8)
    d = torch.frombuffer(bytearray(file), dtype=torch.uint8).to(gpu)
    h = torch.tensor(handles, dtype=torch.int64, device=gpu)
    LT.seal_blocks(d, h, torch.from_numpy(types).to(gpu))
    sealed = d.cpu().numpy().tobytes()
    want = _oracle_seal(file, handles, types.tolist())
    assert sealed == want
    st, crc = LT.verify_blocks(d, h, out_crc=True)
    assert st.cpu().numpy().tolist() == [0] * len(handles)
    for (o, sz), c in zip(handles, crc.cpu().numpy().view(np.uint32).tolist()):
        assert c == W.value(want[o:o + sz + 1])
    assert all(T.verify_block(want, T.BlockHandle(o, sz)) == 0 for o, sz in handles)


@pytest.mark.gpu
def test_gpu_verify_detects_corruption_and_range(gpu):
    import torch
    from lvgpu import table as LT
    rng = np.random.default_rng(72)
    file, handles = _make_table(rng, 200, sizes=rng.integers(0, 9000, size=200))
    sealed = bytearray(_oracle_seal(file, handles, [0] * len(handles)))
    hit = sorted(set(int(x) for x in rng.integers(0, len(handles), size=40)))
    for k in hit:  # flip a byte inside contents, type or stored crc
        o, sz = handles[k]
        sealed[o + int(rng.integers(0, sz + 5))] ^= 0x40
    extra = [(len(sealed) - 4, 0), (len(sealed) - 5, 0), (2**63, 10), (0, 2**40), (10, 2**64 - 1)]
    allh = handles + extra
    want = [T.verify_block(bytes(sealed), T.BlockHandle(o, s)) for o, s in allh]
    assert [want[k] for k in hit] == [1] * len(hit)
    # past the end, a 5-byte window that is not a trailer, offset/size overflow
    assert want[-5:] == [2, 1, 2, 2, 2]
    d = torch.frombuffer(bytearray(sealed), dtype=torch.uint8).to(gpu)
    h = torch.tensor(np.array(allh, dtype=np.uint64).view(np.int64), device=gpu)
    got = LT.verify_blocks(d, h).cpu().numpy().tolist()
    assert got == want
    assert LT.verify_blocks_host(bytes(sealed), np.array(allh, dtype=np.uint64)).tolist() == want
    # the host path reuses the device's cached arena and scratch: a second
    # call of the same size allocates nothing
    import lvgpu
    before = lvgpu.device_counters(0)["allocs"]
    assert LT.verify_blocks_host(bytes(sealed), np.array(allh, dtype=np.uint64)).tolist() == want
    assert lvgpu.device_counters(0)["allocs"] == before


@pytest.mark.gpu
def test_gpu_trailer_fixture(gpu, tfix, arena):
    """Seal arena slices copied into a table and compare with the fixture trailers."""
    import torch
    from lvgpu import table as LT
    parts, handles, types, pos = [], [], [], 0
    for off, ln, ctype, _ in tfix["trailers"]:
        parts.append(arena[off:off + ln] + bytes(5))
        handles.append((pos, ln))
        types.append(ctype)
        pos += ln + 5
    d = torch.frombuffer(bytearray(b"".join(parts)), dtype=torch.uint8).to(gpu)
    LT.seal_blocks(d, torch.tensor(handles, dtype=torch.int64, device=gpu),
                   torch.tensor(types, dtype=torch.uint8, device=gpu))
    out = d.cpu().numpy().tobytes()
    for (o, ln), (_, _, _, hx) in zip(handles, tfix["trailers"]):
        assert out[o + ln:o + ln + 5].hex() == hx


@pytest.mark.gpu
def test_gpu_table_one_launch_any_order(gpu):
    """Seal and verify are one kernel launch that walks the handles in the
    order given (no length sort): shuffled handles, sizes 0-70,000 B mixed
    (several rows-per-round shapes in one wave), a count that is not a
    multiple of the 4 blocks of a wave round, random types, crc output."""
    import lvgpu
    import torch
    from lvgpu import table as LT
    rng = np.random.default_rng(73)
    sizes = np.concatenate([rng.integers(0, 70000, size=150), rng.integers(4000, 4400, size=151), [0, 1, 2, 3, 4]])
    file, handles = _make_table(rng, sizes.size, sizes=sizes)
    perm = rng.permutation(len(handles))
    handles = [handles[i] for i in perm]
    types = rng.integers(0, 256, size=len(handles)).astype(np.uint8)
    d = torch.frombuffer(bytearray(file), dtype=torch.uint8).to(gpu)
    h = torch.tensor(handles, dtype=torch.int64, device=gpu)
    LT.seal_blocks(d, h, torch.from_numpy(types).to(gpu))
    assert lvgpu.last_kernel() == "sst_blocks_kernel<seal>"
    want = _oracle_seal(file, handles, types.tolist())
    assert d.cpu().numpy().tobytes() == want
    st, crc = LT.verify_blocks(d, h, out_crc=True)
    assert lvgpu.last_kernel() == "sst_blocks_kernel<verify,crc>"
    assert st.cpu().numpy().tolist() == [0] * len(handles)
    got = crc.cpu().numpy().view(np.uint32).tolist()
    assert got == [W.value(want[o:o + sz + 1]) for o, sz in handles]
    st = LT.verify_blocks(d, h)  # status only: the two-word staging
    assert lvgpu.last_kernel() == "sst_blocks_kernel<verify>"
    assert st.cpu().numpy().tolist() == [0] * len(handles)


@pytest.mark.gpu
def test_gpu_seal_without_types(gpu):
    """Seal with no per-block types (all 0, the bench's case): the walk parks
    each trailer's file offset instead of its block index, so the flush stores
    without re-reading the handle.  Shuffled handles, sizes 0-70,000 B, a
    count that is not a multiple of 4, and out-of-range handles (skipped)."""
    import torch
    from lvgpu import table as LT
    rng = np.random.default_rng(74)
    sizes = np.concatenate([rng.integers(0, 70000, size=120), rng.integers(4000, 4400, size=201), [0, 1, 2, 3, 4]])
    file, handles = _make_table(rng, sizes.size, sizes=sizes)
    perm = rng.permutation(len(handles))
    handles = [handles[i] for i in perm]
    want = _oracle_seal(file, handles, [0] * len(handles))
    extra = [(len(file) - 4, 0), (2**63, 10), (0, 2**40)]
    d = torch.frombuffer(bytearray(file), dtype=torch.uint8).to(gpu)
    h = torch.tensor(np.array(handles + extra, dtype=np.uint64).view(np.int64), device=gpu)
    LT.seal_blocks(d, h)
    assert d.cpu().numpy().tobytes() == want
    assert LT.verify_blocks(d, h).cpu().numpy().tolist() == [0] * len(handles) + [2, 2, 2]


@pytest.mark.gpu
@pytest.mark.parametrize("shift", [0, 3, 200])
def test_gpu_table_file_order(gpu, shift):
    """Blocks that follow each other (the bench's layout: 4096 + U[0, 256) B
    blocks with their 5-B trailers, in file order, walked in runs of four per
    group) with the file at an offset from a 256-B boundary, a block count that is
    not a multiple of a claim's 16, runs broken by a long block, a short one
    and an out-of-range handle, and corrupted bytes: seal == oracle, verify
    statuses (mismatch exactly where corrupted) and CRCs == oracle."""
    import lvgpu
    import torch
    from lvgpu import table as LT
    rng = np.random.default_rng(75 + shift)
    sizes = rng.integers(4096, 4352, size=203)
    sizes[50], sizes[51], sizes[120] = 70000, 17, 1023
    file, handles = _make_table(rng, sizes.size, sizes=sizes)
    types = rng.integers(0, 4, size=len(handles)).astype(np.uint8)
    want = _oracle_seal(file, handles, types.tolist())
    buf = torch.zeros(len(file) + 512, dtype=torch.uint8, device=gpu)
    base = (256 - buf.data_ptr() % 256) % 256 + shift
    d = buf[base:base + len(file)]
    d.copy_(torch.frombuffer(bytearray(file), dtype=torch.uint8).to(gpu))
    hl = handles[:130] + [(2**62, 5)] + handles[130:]
    h = torch.tensor(np.array(hl, dtype=np.uint64).view(np.int64), device=gpu)
    tl = np.concatenate([types[:130], [0], types[130:]]).astype(np.uint8)
    LT.seal_blocks(d, h, torch.from_numpy(tl).to(gpu))
    assert lvgpu.last_kernel() == "sst_blocks_kernel<seal>"
    assert d.cpu().numpy().tobytes() == want
    bad = sorted(int(x) for x in rng.choice(len(handles), size=12, replace=False))
    for k in bad:
        o, sz = handles[k]
        d[o + int(rng.integers(0, sz + 1))] ^= 0x5A  # contents or the type byte
    st, crc = LT.verify_blocks(d, h, out_crc=True)
    st = st.cpu().numpy().tolist()
    exp = [1 if k in bad else 0 for k in range(len(handles))]
    assert st == exp[:130] + [2] + exp[130:]
    host = d.cpu().numpy().tobytes()
    got = crc.cpu().numpy().view(np.uint32).tolist()
    assert got == [W.value(host[o:o + sz + 1]) for o, sz in handles[:130]] + [0] + \
        [W.value(host[o:o + sz + 1]) for o, sz in handles[130:]]
