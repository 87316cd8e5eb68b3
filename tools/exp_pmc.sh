#!/bin/bash
# PMC counter sets for the CRC kernels of one bench configuration.
#   tools/exp_pmc.sh OUT VARIANT|default [bench args]
set -o pipefail
out=$1; v=$2; shift 2
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$root/$out"
export TMPDIR=/tmp
lib=""
[ "$v" != default ] && lib=$root/leveldb-rs_amd/lib/variants/liblvgpu_$v.so
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  (cd /tmp && LVGPU_EXPERIMENT=1 LVGPU_LIB=$lib timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d "$root/$out/p$i" -o pmc -- \
     python3 "$root/bench.py" --steps 5 --warmup 20 --cpu-seconds 0 --traffic off "$@") > "$root/$out/p$i.txt" 2>&1 || { echo "pass $i failed"; tail -5 "$root/$out/p$i.txt"; exit 1; }
done
python3 - "$root/$out" <<'PY'
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
