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
