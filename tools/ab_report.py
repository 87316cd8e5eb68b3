#!/usr/bin/env python3
"""Summarise a tools/ab_lib.sh directory: frac per workload, product vs variant."""
import glob
import json
import os
import sys


def frac(path):
    with open(path) as f:
        lines = [l for l in f if l.startswith("{")]
    if not lines:
        return None
    d = json.loads(lines[-1])
    if "roofline" in d and d["roofline"] and d["roofline"].get("frac") is not None:
        return d["roofline"]["frac"]
    if "verify" in d:
        return (d["seal"]["frac_of_8TBps"], d["verify"]["frac_of_8TBps"])
    return None


def main(d):
    rows = {}
    for p in sorted(glob.glob(os.path.join(d, "*.json"))):
        if os.path.basename(p).count("_") != 2:
            continue
        tag, w, r = os.path.basename(p)[:-5].split("_")
        rows.setdefault(w, {}).setdefault(tag, []).append(frac(p))
    for w, v in rows.items():
        print(w)
        for tag, fr in sorted(v.items()):
            print(f"   {tag:8s} {fr}")


if __name__ == "__main__":
    main(sys.argv[1])
