"""Steady-state per-kernel durations from a rocprofv3 kernel trace.

    python tools/kstats_steady.py TRACE.csv LAST [OUT.json]

rocprofv3's --stats table averages every launch of a kernel, including the
bench's warmup launches (MI355X clocks take ~60 back-to-back 1 GiB launches to
settle).  bench.py's roofline.achieved is the mean over the K event-timed
launches at the end of the run, so this reports, per lvk:: kernel, the mean,
median and min of its LAST `LAST` launches -- the figure to compare with it.
"""
import collections
import csv
import json
import sys


def main():
    path, last = sys.argv[1], int(sys.argv[2])
    per = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if ("lvk::" in name or "lvh::" in name) and "fill_" not in name:
                per[name.split("(")[0].replace("void ", "")].append(
                    (int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0))
    out = {}
    for name, v in per.items():
        v.sort()
        d = sorted(x for _, x in v[-last:])
        out[name] = {"launches_total": len(v), "launches_used": len(d), "mean_us": round(sum(d) / len(d), 2),
                     "median_us": round(d[len(d) // 2], 2), "min_us": round(d[0], 2), "max_us": round(d[-1], 2)}
    text = json.dumps(out, indent=1)
    print(text)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
