"""the library's static teardown makes no HIP call.

A process that used liblvgpu.so exits with the library's per-device contexts
(g_dev, context.hip), stream workspaces, host-path streams, events and pinned
staging still alive: they are owned by plain pointers and handles, and no
destructor of a static object calls the runtime (a call there would run after
or during the HIP runtime's own teardown -- the round-5 record of a SIGSEGV
in __cxa_finalize under rocprofv3 came from a backed-out path's CU-masked
streams).  tests/teardown/hipspy.c interposes the HIP entry points
the library calls and reports any call liblvgpu.so makes after Python's exit
hooks; a positive control shows the interposer sees the library's calls."""
import os
import re
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _spy(tmp_path):
    so = str(tmp_path / "libhipspy.so")
    subprocess.run(["gcc", "-shared", "-fPIC", "-O1", "-o", so, os.path.join(HERE, "teardown", "hipspy.c"), "-ldl"],
                   check=True, capture_output=True, timeout=120)
    return so


def _run(so, mode, *extra):
    r = subprocess.run([sys.executable, os.path.join(HERE, "teardown", "exit_run.py"), so, mode, *extra],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    ctl = re.search(r"positive_control (\d+)", r.stdout)
    rep = re.search(r"hipspy: calls_from_lvgpu=(\d+) calls_after_exit=(\d+) \[(.*)\]", r.stderr)
    assert ctl and rep, (r.stdout[-2000:], r.stderr[-2000:])
    return int(ctl.group(1)), int(rep.group(2)), rep.group(3)


def test_static_teardown_makes_no_hip_call(tmp_path):
    """CPU: the interposer sees lv_host_alloc reach the runtime (positive
    control; with no device it fails, so there is nothing to free) and nothing
    from the library after exit begins."""
    seen, late, names = _run(_spy(tmp_path), "cpu")
    assert seen >= 1, seen
    assert late == 0, names


def test_interposer_catches_a_static_destructor_calling_hip(tmp_path):
    """Negative control: a library named like the product whose static
    object's destructor calls hipFree is reported."""
    so = _spy(tmp_path)
    bad = str(tmp_path / "liblvgpu_badprobe.so")
    subprocess.run(["g++", "-shared", "-fPIC", "-O1", "-o", bad, os.path.join(HERE, "teardown", "bad_static.cc")],
                   check=True, capture_output=True, timeout=120)
    _, late, names = _run(so, "bad", bad)
    assert late == 1 and "hipFree" in names, (late, names)


@pytest.mark.gpu
def test_static_teardown_makes_no_hip_call_gpu(gpu, tmp_path):
    """GPU: the same after the host paths left library-owned streams, events,
    pinned staging and device buffers alive (batch_host, a pipelined WAL scan
    and its Reader)."""
    seen, late, names = _run(_spy(tmp_path), "gpu")
    assert seen >= 4, seen
    assert late == 0, names
