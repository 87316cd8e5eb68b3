#!/bin/bash
# Where does the sorted walk's per-round time go?  Builds experiment variants
# that drop one piece of per-round work each (wrong CRCs: timing only) and
# times the SST trailer bench and C2/C3 through the offsets API under each.
#   tools/exp_walk.sh OUT
set -e
out=$1
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
vars="notail:-DLVK_EXP_NOTAIL=1 nofix:-DLVK_EXP_NOFIX=1 nomerge:-DLVK_EXP_NOMERGE=1 none3:-DLVK_EXP_NOTAIL=1,-DLVK_EXP_NOFIX=1,-DLVK_EXP_NOMERGE=1"
for spec in $vars; do
  name=${spec%%:*}; flags=${spec#*:}
  bash tools/build_variant.sh "$name" ${flags//,/ } > "$out/build_$name.txt" 2>&1
done
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --table > "$out/prod_table_$r.json" 2>> "$out/err.txt"
  for w in c2 c3; do
    timeout -k 10 200 python3 bench.py --workload $w --api offsets --cpu-seconds 0 --traffic off > "$out/prod_${w}_$r.json" 2>> "$out/err.txt"
  done
  for spec in $vars; do
    name=${spec%%:*}
    lib=$root/leveldb-rs_amd/lib/variants/liblvgpu_$name.so
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$lib timeout -k 10 200 python3 bench.py --table > "$out/${name}_table_$r.json" 2>> "$out/err.txt"
    for w in c2 c3; do
      LVGPU_EXPERIMENT=1 LVGPU_LIB=$lib timeout -k 10 200 python3 bench.py --workload $w --api offsets --cpu-seconds 0 --traffic off > "$out/${name}_${w}_$r.json" 2>> "$out/err.txt"
    done
  done
done
echo walk done
