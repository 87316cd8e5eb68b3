"""Summary table of one tools/measure_round.sh pass.

    python tools/round_summary.py OUTDIR  > OUTDIR/summary.md

Every offsets-API line is reported twice: the HIP-event mean per call
(bench.py roofline.kernel_ms_avg) and the sum of the call's kernels' steady
rocprofv3 means (prof_<w>_steady.json: the last 50 launches of each kernel),
with the fraction of 8 TB/s each gives (quote both)."""
import glob
import json
import os
import sys

PEAK = 8e12


def load(path):
    try:
        with open(path) as f:
            for line in f:
                line = line.strip()
                if line.startswith("{"):
                    last = json.loads(line)
            return last
    except (OSError, ValueError, UnboundLocalError):
        return None


def ksum(path):
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        d = None
    if not d:
        return None, {}
    d = {k: v for k, v in d.items() if v["launches_total"] >= 10}  # not the one-off parity-check launches
    return sum(v["mean_us"] for v in d.values()), {k.split("::")[-1]: v["mean_us"] for k, v in d.items()}


def main():
    out = sys.argv[1]
    rows = ["| line | events | rocprof kernel sum | notes |", "|---|---|---|---|"]
    for name, prof in (("default_driver", "c3"), ("default", "c3"), ("c3_offsets", None), ("c2", "c2"),
                       ("c4", "c4"), ("c5", None), ("c5_strong", None)):
        d = load(os.path.join(out, name + ".json"))
        if not d:
            continue
        rf = d["roofline"]
        nb = rf["bytes_per_launch"]
        ev = f"{rf['kernel_ms_avg'] * 1e3:.1f} us, frac {rf['frac']:.4f}"
        ks, parts = ksum(os.path.join(out, f"prof_{prof}_steady.json")) if prof else (None, {})
        kt = f"{ks:.1f} us, frac {nb / (ks * 1e-6) / PEAK:.4f}" if ks else "-"
        note = f"value {d['value']} GiB/s; traffic {rf['traffic'] / nb:.4f}x" if rf.get("traffic") else \
            f"value {d['value']} GiB/s"
        if parts:
            note += "; " + ", ".join(f"{k.split('(')[0]} {v}" for k, v in parts.items())
        rows.append(f"| {name} | {ev} | {kt} | {note} |")
    t = load(os.path.join(out, "table.json"))
    if t:
        rows.append(f"| table seal / verify | {t['seal']['ms_avg'] * 1e3:.1f} / {t['verify']['ms_avg'] * 1e3:.1f} us, "
                    f"frac {t['seal']['frac_of_8TBps']} / {t['verify']['frac_of_8TBps']} | - | |")
    h = load(os.path.join(out, "hash.json"))
    if h:
        rows.append(f"| hash | {h['ms_avg'] * 1e3:.1f} us, frac {h['frac_of_8TBps']} | - | {h['value']} Gkeys/s |")
    w = load(os.path.join(out, "wal_device.json"))
    if w:
        ks, parts = ksum(os.path.join(out, "prof_wal_steady.json"))
        kt = f"{ks:.1f} us, frac {w['log_bytes'] / (ks * 1e-6) / PEAK:.4f}" if ks else "-"
        rows.append(f"| WAL device scan | {w['roofline']['ms_avg'] * 1e3:.1f} us, frac {w['roofline']['frac']} | {kt} | "
                    + ", ".join(f"{k.split('(')[0]} {v}" for k, v in parts.items()) + " |")
    lg = load(os.path.join(out, "long.json"))
    if lg:
        for r in lg["results"]:
            med = lambda a: f" (median {r[a]['us_p50']})" if "us_p50" in r[a] else ""
            rows.append(f"| {r['blocks']} x {r['block_bytes']} B | strided {r['strided']['us_avg']} us{med('strided')}, "
                        f"offsets {r['offsets']['us_avg']} us{med('offsets')} | - | {r['offsets']['kernels']} |")
    g = load(os.path.join(out, "gloo2.json"))
    if g:
        rows.append(f"| N=2 launcher (gloo, 1 GPU) | {g['value']} GiB/s | - | n_gpus {g['n_gpus']}, world {g['world_size']}, "
                    f"{g['launcher']} |")
    print("\n".join(rows))
    for f in sorted(glob.glob(os.path.join(out, "prof8f", "*_pmc.json"))):
        print(f"\n{os.path.basename(f)}: " + json.dumps(json.load(open(f))))


if __name__ == "__main__":
    main()
