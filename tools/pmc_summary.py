"""Per-kernel HBM bytes per launch from rocprofv3 --pmc passes.

    python tools/pmc_summary.py DIR [OUT.json]

Reads every */**/*counter_collection.csv under DIR (one counter per pass:
FETCH_SIZE or WRITE_SIZE, in KiB) and reports, per lvk:: kernel, the mean
over its launches in bytes.  FETCH_SIZE is doubled: on gfx950 it counts half
the bytes of a 16-B-per-lane streaming read (MI355X_MICROARCH.md, HBM);
WRITE_SIZE is exact for 16-B-per-lane stores and uncalibrated for narrower
ones (the SST seal's 5-byte trailers), so it is reported as read."""
import collections
import csv
import glob
import json
import os
import sys

SCALE = {"FETCH_SIZE": 2.0 * 1024.0, "WRITE_SIZE": 1024.0}


def main():
    root = sys.argv[1]
    per = collections.defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                ctr = row.get("Counter_Name", "")
                if ("lvk::" in name or "lvh::" in name) and "fill_" not in name and ctr in SCALE:
                    short = name.split("(")[0].replace("void ", "")
                    per[(short, ctr)].append(float(row["Counter_Value"]) * SCALE[ctr])
    out = {}
    for (k, c), v in sorted(per.items()):
        out.setdefault(k, {})[c] = {"bytes_per_launch_mean": round(sum(v) / len(v)), "launches": len(v),
                                    "min": round(min(v)), "max": round(max(v))}
    text = json.dumps(out, indent=1)
    print(text)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fh:
            fh.write(text + "\n")


if __name__ == "__main__":
    main()
