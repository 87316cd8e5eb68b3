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
        if d.get("cpu_baseline"):
            note += f"; cpu {d['cpu_baseline']['value']} GiB/s (1 core)"
        rows.append(f"| {name} | {ev} | {kt} | {note} |")
        c5 = d.get("c5_strong")
        if c5:
            rows.append(f"| {name}: c5_strong sub-record | {c5['ms_per_step']} ms per 64 GiB step, frac "
                        f"{c5['hbm_peak_frac']} | - | value {c5['value']} GiB/s (barrier-inclusive "
                        f"{c5['value_barrier_inclusive']}), n_gpus {c5['n_gpus']} |")
    t = load(os.path.join(out, "table.json"))
    if t:
        cpu = t.get("cpu_baseline") or {}
        cn = (f"cpu verify / seal {cpu['verify']['value']} / {cpu['seal']['value']} GiB/s (1 core)" if cpu else "")
        he = t.get("host_e2e") or {}
        if he:
            cn += f"; lv_sst_verify_blocks_host {he['pageable']['GiB_per_s']} / {he['pinned']['GiB_per_s']} GiB/s"
        rows.append(f"| table seal / verify | {t['seal']['ms_avg'] * 1e3:.1f} / {t['verify']['ms_avg'] * 1e3:.1f} us, "
                    f"frac {t['seal']['frac_of_8TBps']} / {t['verify']['frac_of_8TBps']} | - | {cn} |")
    h = load(os.path.join(out, "hash.json"))
    if h:
        fr = h["roofline"]["frac"] if "roofline" in h else h.get("frac_of_8TBps")
        note = f"{h['value']} Gkeys/s"
        for k in ("packed_u64", "packed_u32"):
            if k in h:
                note += f"; {k} {h[k]['ms_avg'] * 1e3:.1f} us, frac {h[k]['roofline']['frac']}"
        hb = h.get("roofline_hbm") or {}
        if "frac_all_bytes" in hb:
            note += f"; all bytes moved frac {hb['frac_all_bytes']}"
        if h.get("roofline_valu"):
            note += f"; VALU issue frac {h['roofline_valu']['frac']}"
        if h.get("cpu_baseline"):
            note += f"; cpu {h['cpu_baseline']['value']} Gkeys/s (1 core)"
        rows.append(f"| hash (key bytes) | {h['ms_avg'] * 1e3:.1f} us, frac {fr} | - | {note} |")
    w = load(os.path.join(out, "wal_device.json"))
    if w:
        ks, parts = ksum(os.path.join(out, "prof_wal_steady.json"))
        kt = f"{ks:.1f} us, frac {w['log_bytes'] / (ks * 1e-6) / PEAK:.4f}" if ks else "-"
        cn = f"; cpu {w['cpu_baseline']['value']} GB/s (1 core)" if w.get("cpu_baseline") else ""
        rows.append(f"| WAL device scan | {w['roofline']['ms_avg'] * 1e3:.1f} us, frac {w['roofline']['frac']} | {kt} | "
                    + ", ".join(f"{k.split('(')[0]} {v}" for k, v in parts.items()) + cn + " |")
    wl = load(os.path.join(out, "wal.json"))
    if wl:
        rn = wl.get("reader_native") or {}
        rows.append(f"| WAL host (encode / scan{' / native reader' if rn else ''}) | {wl['encode']['GiB_per_s']} / "
                    f"{wl['scan']['GiB_per_s']}{' / ' + str(rn['GiB_per_s']) if rn else ''} GiB/s | - | "
                    + (f"scan + reader {wl['scan_plus_native_reader']['GiB_per_s']} GiB/s" if rn else "") + " |")
    lg = load(os.path.join(out, "long.json"))
    if lg:
        for r in lg["results"]:
            med = lambda a: f" (median {r[a]['us_p50']})" if "us_p50" in r[a] else ""
            hn = (f", hinted {r['offsets_hint']['us_avg']} us{med('offsets_hint')} ({r['offsets_hint']['kernels']})"
                  if "offsets_hint" in r else "")
            rows.append(f"| {r['blocks']} x {r['block_bytes']} B | strided {r['strided']['us_avg']} us{med('strided')}, "
                        f"offsets {r['offsets']['us_avg']} us{med('offsets')}{hn} | - | {r['offsets']['kernels']} |")
    va = load(os.path.join(out, "variants.json"))
    if va:
        for r in va["results"]:
            rows.append(f"| variant {r['variant']} | {r['ms_avg'] * 1e3:.1f} us, frac {r['frac_of_8TBps']} | - | "
                        f"{r['GiB_per_s']} GiB/s; {r['kernels']} |")
    g = load(os.path.join(out, "gloo2.json"))
    if g:
        c5 = g.get("c5_strong") or {}
        rows.append(f"| N=2 launcher (gloo, 1 GPU) | {g['value']} GiB/s | - | n_gpus {g['n_gpus']}, world {g['world_size']}, "
                    f"{g['launcher']}" + (f"; c5_strong {c5['value']} GiB/s, {len(c5['per_gpu'])} ranks" if c5 else "")
                    + " |")
    print("\n".join(rows))
    for f in sorted(glob.glob(os.path.join(out, "prof8f", "*_pmc.json"))):
        print(f"\n{os.path.basename(f)}: " + json.dumps(json.load(open(f))))


if __name__ == "__main__":
    main()
