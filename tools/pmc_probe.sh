#!/bin/bash
# PMC passes over an arbitrary command; summarises counters per kernel name.
# usage: tools/pmc_probe.sh OUTDIR KERNEL_SUBSTR -- cmd args...
set -o pipefail
out=$1; shift; ksub=$1; shift; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $set --output-format csv -d "$out/p$i" -o pmc -- "$@" > "$out/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$out/p$i.log"; }
done
python3 - "$out" "$ksub" <<'PY'
import csv, glob, os, sys, collections
out, ksub = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")
        if ksub in k:
            agg[k[:90]][row["Counter_Name"]].append(float(row["Counter_Value"]))
with open(os.path.join(out, "summary.txt"), "w") as fo:
    for k in sorted(agg):
        print(k); fo.write(k + "\n")
        for c in sorted(agg[k]):
            v = sorted(agg[k][c]); line = f"   {c:24s} median {v[len(v)//2]:.6g} n={len(v)}"
            print(line); fo.write(line + "\n")
PY
