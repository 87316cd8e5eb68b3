#!/bin/bash
# Collect rocprofv3 PMC counters for the CRC kernel, one small counter set per
# pass (kernel dispatch counters only; never combined with sys/runtime traces).
# usage: tools/pmc_passes.sh OUTDIR [bench args...]
set -o pipefail
out=$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $set --output-format csv -d "$out/p$i" -o pmc -- python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --traffic off --no-settle "$@" > "$out/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$out/p$i.log"; }
done
python3 - "$out" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "")
        if "lvk::" in name and "fill_" not in name:
            short = name.split("(")[0].replace("void ", "")
            agg[(short, row["Counter_Name"])].append(float(row["Counter_Value"]))
with open(os.path.join(out, "summary.txt"), "w") as fo:
    for k in sorted(agg):
        v = sorted(agg[k]); line = f"{k[0]:44s} {k[1]:24s} median {v[len(v)//2]:.6g}  n={len(v)}"
        print(line); fo.write(line + "\n")
PY
