#!/bin/bash
# Round 5: what the SQ instruction counters count on gfx950 (tools/pmc_calib:
# known VALU / SALU counts per wave), then the same counters over the hash
# bench's kernels -- the VALU-issue side of the hash roofline.
# usage: tools/r05_valu.sh OUTDIR
set -o pipefail
out=$(realpath -m "${1:-gpurun_out/r05v}")
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -k 10 60 "$root/tools/pmc_calib" > "$out/calib_timed.json" 2>&1 && cat "$out/calib_timed.json" &&
timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d "$out/calib" -o pmc -- "$root/tools/pmc_calib" \
  > "$out/calib.log" 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$out/hash" -o pmc -- python3 "$root/bench.py" --hash \
  --steps 3 --warmup 1 --cpu-seconds 0 > "$out/hash.log" 2>&1 &&
python3 - "$out" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "").split("(")[0].replace("void ", "")
        if "valu_calib" in name or "hash_kernel" in name:
            agg[(name, row["Counter_Name"])].append(float(row["Counter_Value"]))
with open(os.path.join(out, "summary.txt"), "w") as fo:
    for k in sorted(agg):
        v = sorted(agg[k]); line = f"{k[0]:52s} {k[1]:22s} median {v[len(v)//2]:.6g}  n={len(v)}"
        print(line); fo.write(line + "\n")
PY
# the counter CSVs are large (one row per launch and counter): keep the summary only
rm -rf "$out/calib" "$out/hash"
