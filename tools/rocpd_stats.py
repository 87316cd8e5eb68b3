#!/usr/bin/env python3
"""Per-kernel duration stats from a rocprofv3 rocpd database (ROCm 7's default
output of `rocprofv3 --kernel-trace --stats` without --output-format csv).

    python tools/rocpd_stats.py RESULTS.db OUT.json [LAST]

For every lvk:: kernel: launches, mean / median / min / max over all launches
(rocprofv3's --stats figure) and the mean of the LAST launches (default 20:
the bench's event-timed pass, the figure roofline.achieved is compared with).
"""
import json
import sqlite3
import statistics
import sys


def main():
    db, out_path = sys.argv[1], sys.argv[2]
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    c = sqlite3.connect(db)
    per = {}
    for name, dur in c.execute("select name, duration from kernels order by start"):
        if "lvk::" in name:
            per.setdefault(name.split("(")[0].replace("void ", ""), []).append(dur / 1000.0)
    out = {}
    for name, v in per.items():
        tail = v[-last:]
        out[name] = {"launches": len(v), "mean_us_all": round(sum(v) / len(v), 2),
                     "median_us_all": round(statistics.median(v), 2), "min_us": round(min(v), 2),
                     "max_us": round(max(v), 2), f"mean_us_last{last}": round(sum(tail) / len(tail), 2)}
    with open(out_path, "w") as f:
        json.dump({"source": db, "kernels": out}, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
