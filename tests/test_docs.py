"""INTEGRATION.md binds every entry point include/lvgpu/*.h declares (the
drop-in boundary a Rust maintainer wires up), and names no entry point the
headers do not declare."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "lvgpu", "*.h")):
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b(lv_[a-z0-9_]+)\s*\(", src))
    return names


def test_integration_binds_every_declared_entry_point():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    bound = set(re.findall(r"\bfn (lv_[a-z0-9_]+)\s*\(", doc))
    missing = sorted(_declared() - set(re.findall(r"\b(lv_[a-z0-9_]+)", doc)))
    assert not missing, missing
    stale = sorted(bound - _declared())
    assert not stale, stale


def test_design_evidence_paths_exist():
    """Every evidence directory DESIGN.md, README.md and HISTORY.md cite exists: full
    `profiles/rNN/<dir>/` paths, and the bare `<dir>/` names the round
    tables use for a directory under some round's profiles (or one level
    below, e.g. final/recovery5/)."""
    text = "".join(open(os.path.join(ROOT, f)).read() for f in ("DESIGN.md", "README.md", "HISTORY.md"))
    full = set(re.findall(r"profiles/(r\d\d)/([A-Za-z0-9_]+)/", text))
    missing = sorted(f"profiles/{r}/{d}/" for r, d in full if not os.path.isdir(os.path.join(ROOT, "profiles", r, d)))
    assert not missing, missing
    dirs = {os.path.basename(p.rstrip("/")) for p in glob.glob(os.path.join(ROOT, "profiles", "r*", "*", ""))}
    dirs |= {os.path.basename(p.rstrip("/")) for p in glob.glob(os.path.join(ROOT, "profiles", "r*", "*", "*", ""))}
    top = {"oracle", "profiles", "tests", "tools", "include", "leveldb-rs_amd"}
    bare = set(re.findall(r"`([a-z0-9_]+)/`", text)) - top
    unresolved = sorted(bare - dirs)
    assert not unresolved, unresolved
