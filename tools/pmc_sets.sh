#!/bin/bash
# rocprofv3 PMC passes with caller-chosen counter sets (one pass each, kernel
# dispatch counters only), summarised per lvk:: kernel.
#   tools/pmc_sets.sh OUTDIR "SET1" "SET2" ... -- [bench args]
set -o pipefail
out=$(realpath -m "$1"); shift
sets=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do sets+=("$1"); shift; done
[ "$1" = "--" ] && shift
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$out/p$i" -o pmc -- python3 "$root/bench.py" --steps 5 --warmup 1 --cpu-seconds 0 --traffic off --no-settle "$@" > "$out/p$i.log" 2>&1 || { echo "pass $i ($set) failed"; tail -3 "$out/p$i.log"; }
done
python3 - "$out" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "")
        if ("lvk::" in name or "lvh::" in name) and "fill_" not in name:
            short = name.split("(")[0].replace("void ", "")
            agg[(short, row["Counter_Name"])].append(float(row["Counter_Value"]))
with open(os.path.join(out, "summary.txt"), "w") as fo:
    for k in sorted(agg):
        v = sorted(agg[k]); line = f"{k[0]:44s} {k[1]:24s} median {v[len(v)//2]:.6g}  n={len(v)}"
        print(line); fo.write(line + "\n")
PY
