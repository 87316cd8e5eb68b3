"""C-ABI checks that need no GPU: liblvgpu.so loads, exports every symbol that
include/lvgpu/crc32c.h declares, and the host scalar drop-ins (crc32c.rs
value/extend/mask/unmask/extend_sw/extend_hw) agree with the golden vectors."""
import ctypes
import os
import subprocess

import pytest

from conftest import ROOT, kat_bytes
import lvgpu


def test_library_builds():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "leveldb-rs_amd")], check=True)
    assert os.path.exists(lvgpu.LIB_PATH)


def test_exports_every_declared_symbol():
    names = lvgpu.declared_symbols()
    assert len(names) >= 13
    L = ctypes.CDLL(lvgpu.LIB_PATH)
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert "lv_crc32c_batch_device" in names and "lv_crc32c_value" in names


def test_nm_exports_are_c_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", lvgpu.LIB_PATH], capture_output=True, text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    for n in lvgpu.declared_symbols():
        assert n in syms, n  # unmangled: extern "C"


def test_scalar_kats(kat):
    for k in kat["kats"]:
        d = kat_bytes(k)
        assert lvgpu.value(d) == k["value"], k["name"]
        assert lvgpu.extend_sw(0, d) == k["value"], k["name"]
        assert lvgpu.extend_hw(0, d) == k["value"], k["name"]
        assert lvgpu.mask(k["value"]) == k["masked"]
        assert lvgpu.unmask(k["masked"]) == k["value"]


def test_scalar_properties():
    # crc32c.rs:174-193
    assert lvgpu.value(b"a") != lvgpu.value(b"foo")
    assert lvgpu.value(b"hello world") == lvgpu.extend(lvgpu.value(b"hello "), b"world")
    crc = lvgpu.value(b"foo")
    assert lvgpu.mask(crc) != crc
    assert lvgpu.mask(lvgpu.mask(crc)) != crc
    assert lvgpu.unmask(lvgpu.mask(crc)) == crc
    assert lvgpu.unmask(lvgpu.unmask(lvgpu.mask(lvgpu.mask(crc)))) == crc
    assert lvgpu.extend(0x12345678, b"") == 0x12345678


def test_scalar_golden_cases(kat, arena):
    for off, ln, seed, crc, masked in kat["cases"]:
        d = arena[off:off + ln]
        assert lvgpu.extend(seed, d) == crc
        assert lvgpu.extend_sw(seed, d) == crc


def test_batch_without_gpu_fails_loudly():
    """No CPU fallback: on a machine without a GPU the batch API errors."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    rc = lvgpu.lib().lv_device_init()
    assert rc != 0
    assert lvgpu.lib().lv_last_error()


def test_scalar_combine():
    """lv_crc32c_combine joins the CRCs of a split buffer (an addition for
    callers that cut long buffers): every split point of random buffers,
    seeded, and empty parts."""
    import random
    rng = random.Random(99)
    for _ in range(40):
        d = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 3000)))
        s = rng.getrandbits(32)
        cut = rng.randrange(0, len(d) + 1)
        a, b = d[:cut], d[cut:]
        assert lvgpu.combine(lvgpu.extend(s, a), lvgpu.value(b), len(b)) == lvgpu.extend(s, d)
    assert lvgpu.combine(0x1234, lvgpu.value(b""), 0) == 0x1234
    big = bytes(range(256)) * 4096  # 1 MiB: a long shift
    assert lvgpu.combine(lvgpu.value(b"head"), lvgpu.value(big), len(big)) == lvgpu.value(b"head" + big)


def test_argument_checks_before_any_device_call():
    """Argument validation of the batch entry points happens before they touch
    the GPU, with an error code and a message (no CPU fallback, no crash)."""
    import lvgpu.wal as LW
    L = lvgpu.lib()
    W = LW._bind()
    vp = ctypes.c_void_p
    fake = vp(0x1000)  # never dereferenced: every call below fails its checks first
    # strided: more than 2^32-1 blocks (output slots are 32-bit)
    rc = L.lv_crc32c_batch_strided(fake, 16, 16, 1 << 32, None, fake, 0, None)
    assert rc == -1 and b"2^32" in L.lv_last_error()
    # device WAL scan: null count, misaligned log, workspace too small
    assert W.lv_wal_scan_device(fake, 64, fake, fake, fake, 8, None, fake, 1 << 20, None) == -1
    assert W.lv_wal_scan_device(vp(0x1004), 64, fake, fake, fake, 8, fake, fake, 1 << 20, None) == -1
    assert b"aligned" in L.lv_last_error()
    need = W.lv_wal_scan_workspace_bytes(64, 8)
    assert need > 0
    assert W.lv_wal_scan_device(fake, 64, fake, fake, fake, 8, fake, fake, need - 1, None) == -1
    assert b"workspace" in L.lv_last_error()
    # the workspace grows with the capacity: a 16-B entry, the CRC by sorted
    # position and the sorted position per record (the five-launch layout,
    # which bounds the one-launch scan's at this size)
    assert W.lv_wal_scan_workspace_bytes(64, 2008) - W.lv_wal_scan_workspace_bytes(64, 1008) == 1000 * 24
    # kernel-choice query: empty on a thread that has launched nothing
    import threading
    seen = []
    t = threading.Thread(target=lambda: seen.append(L.lv_crc32c_last_kernel()))
    t.start()
    t.join()
    assert seen == [b""]


def test_workspace_bytes_cover_pieces():
    """The offsets-API workspace holds n sorted entries plus the long-buffer
    split's piece budget, whatever n, and the unsort's two words per buffer."""
    small, big = lvgpu.workspace_bytes(1), lvgpu.workspace_bytes(1 << 20)
    assert small >= 65536 * 16  # the piece entries alone
    # 16-B entry + 4-B seed + the CRC by sorted position + the sorted position, per buffer
    assert big - small >= ((1 << 20) - 1) * 28


CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "leveldb-rs_amd", "csrc")


def _knobs():
    import re
    with open(os.path.join(CSRC, "lvk", "knobs.h")) as f:
        text = f.read()
    guard = text[text.index("#if !defined(LVK_EXPERIMENT_BUILD)"):text.index("#error")]
    return set(re.findall(r"#ifndef (LVK_\w+)", text)), set(re.findall(r"defined\((LVK_\w+)\)", guard))


def test_every_kernel_switch_is_guarded():
    """Every LVK_* switch the kernels read has its default in lvk/knobs.h and
    is refused there outside experiment builds (no product-path
    macro untested at a non-default value)."""
    import glob
    import re
    defaults, guarded = _knobs()
    guarded.discard("LVK_EXPERIMENT_BUILD")
    assert defaults and defaults == guarded
    used = set()
    for path in glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True) + \
            glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cc")):
        with open(path) as f:
            used |= set(re.findall(r"\bLVK_[A-Z0-9_]+\b", f.read()))
    used -= {"LVK_EXPERIMENT_BUILD", "LVK_EXP_"}  # "LVK_EXP_*" in comments
    assert used <= defaults, sorted(used - defaults)


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_product_build_refuses_kernel_switches():
    """A product build with a non-default switch stops at lvk/knobs.h; the
    same define in an experiment build passes the guard."""
    import subprocess
    src = os.path.join(CSRC, "sort.hip")
    base = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-E", "-o", os.devnull, src]
    bad = subprocess.run(base + ["-DLVK_SST_RUN=1"], capture_output=True, text=True, timeout=300)
    assert bad.returncode != 0 and "LVK_* kernel switches" in bad.stderr
    ok = subprocess.run(base + ["-DLVK_SST_RUN=1", "-DLVK_EXPERIMENT_BUILD=1"], capture_output=True, text=True,
                        timeout=300)
    assert ok.returncode == 0, ok.stderr[-2000:]


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_streaming_kernels_do_not_spill():
    """The streaming kernels stay within their register budget: no VGPR spill
    in the unseeded class kernel (C2 / C4 / C3 via offsets / the WAL scan),
    the uniform-block kernels (the headline) or the SST walk.  Round 4 had a
    change put eight selected class bounds in registers: 24 VGPRs of spills,
    C3 via offsets 0.75 -> 0.67 -- a spill reload is a vector memory
    operation, so its wait also waits for every prefetch in flight."""
    import re
    import subprocess
    want = {"classes.hip": ["crc32c_classes_kernelILb0E"], "blocks.hip": ["crc32c_blocks_kernelILi16ELb0ELb0ELb0E"],
            "sst.hip": ["sst_blocks_kernelILb0ELb0E", "sst_blocks_kernelILb1ELb0E"]}
    for src, kernels in want.items():
        r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                            "-munsafe-fp-atomics", "--cuda-device-only", "-c", "-o", os.devnull,
                            os.path.join(CSRC, src), "-Rpass-analysis=kernel-resource-usage"],
                           capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
        spills, name = {}, None
        for line in r.stderr.splitlines():
            m = re.search(r"Function Name: (\S+)", line)
            if m:
                name = m.group(1)
            m = re.search(r"VGPRs Spill: (\d+)", line)
            if m and name:
                spills[name] = int(m.group(1))
        for k in kernels:
            hits = {n: v for n, v in spills.items() if k in n}
            assert hits and all(v == 0 for v in hits.values()), (src, hits)


def test_device_counters_query():
    """lv_device_counters: readable without a GPU (zero before any host-path
    call), bounds-checked, and a short `n` fills only that many slots."""
    import ctypes
    L = lvgpu.lib()
    out = (ctypes.c_uint64 * 4)(7, 7, 7, 7)
    assert L.lv_device_counters(0, ctypes.cast(out, ctypes.c_void_p), 3) == 0
    assert out[3] == 7  # only three counters exist
    out2 = (ctypes.c_uint64 * 2)(9, 9)
    assert L.lv_device_counters(1, ctypes.cast(out2, ctypes.c_void_p), 1) == 0 and out2[1] == 9
    assert L.lv_device_counters(64, ctypes.cast(out, ctypes.c_void_p), 3) != 0
    assert L.lv_device_counters(-1, ctypes.cast(out, ctypes.c_void_p), 3) != 0
    assert L.lv_device_counters(0, None, 3) != 0
    assert L.lv_device_counters(0, None, 0) == 0
    assert set(lvgpu.device_counters(0)) == {"h2d", "d2h", "allocs"}


def _ceil_log2(x):
    return 0 if x <= 1 else (x - 1).bit_length()


def _split_rule(L, total, pmin=12, maxp=4096):
    """lvk::split_rule (csrc/lvk/sort.h) in Python: (pieces, log2 piece length)."""
    if L <= 16384:
        return 0, 0
    q = max(_ceil_log2(total // 16384), _ceil_log2((L + maxp - 1) // maxp), pmin)
    q = min(q, 31)
    if L <= (2 << q):
        return 0, 0
    return (L + (1 << q) - 1) >> q, q


def _needs_join(lens, cus, fused_max=1024, waves=16):
    """Whether the library launches combine_long_kernel: on the sorted path
    (> 1,024 buffers) always -- it also unsorts the class kernel's CRCs --
    but for a uniform batch with nothing to split (the identity list, no
    sort); for a small batch when a split buffer is not joined in place by
    the fused kernel (crc32c_fused_small_kernel's unit layout,
    csrc/classes.hip)."""
    total = sum(lens)
    sp = [_split_rule(L, total) for L in lens]
    if len(lens) > fused_max:
        return not (len(set(lens)) == 1 and not any(m for m, _ in sp))
    if not any(m for m, _ in sp):
        return False
    units = [m if m else 1 for m, _ in sp]
    pre = [0]
    for u in units[:-1]:
        pre.append(pre[-1] + u)
    nunits = sum(units)
    onepass = nunits <= 4 * waves * cus
    S = 4 * ((nunits + 4 * cus - 1) // (4 * cus)) if onepass else 1
    pb = min(max(_ceil_log2(total // 16384), 12), 31)
    for (m, p), pr in zip(sp, pre):
        local = onepass and m and p == pb and pr // S == (pr + m - 1) // S
        if m and not local:
            return True
    return False


def test_hint_join_decision_matches_the_device_layout():
    """lv_crc32c_hint_needs_join (the host half of lv_crc32c_batch_device_hint)
    leaves the join out exactly when the device would find nothing to join:
    uniform batches against a Python replica of split_rule and the fused
    kernel's unit layout; other batches whenever the longest buffer cannot
    split (conservative otherwise)."""
    import random
    L = lvgpu.lib()
    L.lv_crc32c_hint_needs_join.restype = ctypes.c_int
    L.lv_crc32c_hint_needs_join.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
    rng = random.Random(404)
    cases = [(1024, 65536, 256, False), (1, 16 << 20, 256, True), (16, 1 << 20, 256, True), (300, 4096, 256, False),
             (64, 16 << 20, 256, True), (2048, 65536, 256, True), (4096, 16384, 256, False)]
    for _ in range(3000):
        n = rng.choice([1, 2, 3, 7, 16, 64, 100, 255, 256, 512, 1000, 1024, 1025, 4096])
        size = rng.choice([rng.randrange(0, 70000), 1 << rng.randrange(10, 25), rng.randrange(1, 1 << 24)])
        cases.append((n, size, rng.choice([64, 80, 256, 304]), None))
    for n, size, cus, want in cases:
        h = lvgpu.BatchHint(n * size, size, 1)
        got = L.lv_crc32c_hint_needs_join(ctypes.addressof(h), n, cus)
        ref = _needs_join([size] * n, cus)
        assert bool(got) == ref, (n, size, cus)
        if want is not None:
            assert ref == want, (n, size, cus)
    for _ in range(500):  # non-uniform: the sorted path always, small batches iff the longest buffer can split
        n = rng.randrange(1, 3000)
        lens = [rng.randrange(0, 1 << rng.randrange(4, 22)) for _ in range(n)]
        h = lvgpu.hint_for(lens)
        got = L.lv_crc32c_hint_needs_join(ctypes.addressof(h), n, 256)
        assert bool(got) == (n > 1024 or _split_rule(max(lens), sum(lens))[0] > 0)
        assert bool(got) >= _needs_join(lens, 256)  # never leaves out a join the device needs


def _uniform_plan(n, blen, cus):
    """Replica of lvh::uniform_plan (blocks.hip: pick_split, pick_block_gi,
    the fused-join rule) for a 16-B aligned uniform batch: (pieces log2,
    group size or None, scratch bytes)."""
    want = 4 * cus * 16
    ps = 0
    while (n << ps) < want and ps < 12:
        s2 = 2 << ps
        if blen % s2 or (blen // s2) % 1024 or blen // s2 < 4096:
            break
        ps += 1
    if ps:
        nv = n << ps
        fused = (1 << ps) <= 16 and nv <= 64 * cus
        return ps, None, 0 if fused else nv * 4
    if blen == 0:
        return 0, None, 0
    fits = lambda g: blen % (16 * g * 4) == 0
    if n < want and fits(64):
        return 0, 64, 0
    return 0, next((g for g in (16, 4, 1) if fits(g)), None), 0


def test_aligned_hint_join_decision():
    """LV_HINT_ALIGNED16: a uniform batch of whole 1 KiB batches runs on the
    strided API's kernels, whose join (combine_pieces_*) runs only for a split
    whose pieces are not joined in the walk; other lengths keep the unaligned
    decision."""
    import random
    L = lvgpu.lib()
    cases = [(1024, 65536, 0), (1, 16 << 20, 1), (16, 1 << 20, 1), (20000, 4096, 0), (2000, 8192, 0),
             (5000, 4000, 0), (1100, 160 << 10, 1), (600, 1000, 0)]
    for n, size, want in cases:
        h = lvgpu.BatchHint(n * size, size, lvgpu.HINT_UNIFORM | lvgpu.HINT_ALIGNED16)
        assert L.lv_crc32c_hint_needs_join(ctypes.addressof(h), n, 256) == want, (n, size)
    rng = random.Random(808)
    for _ in range(400):
        n = rng.randrange(1, 40000)
        size = rng.choice([1024, 2048, 4096, 8192, 65536, 1 << 20, 3 << 20, 16 << 20, 5000, 40000])
        cus = rng.choice([64, 80, 256, 304])
        h = lvgpu.BatchHint(n * size, size, 3)
        ps, g, scratch = _uniform_plan(n, size, cus)
        got = L.lv_crc32c_hint_needs_join(ctypes.addressof(h), n, cus)
        if ps or g:
            assert got == int(scratch > 0), (n, size, cus)
        else:
            h1 = lvgpu.BatchHint(n * size, size, 1)
            assert got == L.lv_crc32c_hint_needs_join(ctypes.addressof(h1), n, cus), (n, size, cus)
    # hint_for sets the bit only for uniform lengths at 16-B multiples
    assert lvgpu.hint_for([4096] * 3, [0, 4096, 8192]).uniform == 3
    assert lvgpu.hint_for([4096] * 3, [0, 4104, 8192]).uniform == 1
    assert lvgpu.hint_for([4096, 10], [0, 4096]).uniform == 0
