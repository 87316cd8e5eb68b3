#!/bin/bash
# SST trailer bench under the product library and experiment variants, alternated:
#   tools/ab_table.sh OUT "name1:-DFOO=1,-DBAR=2 name2:-DFOO=0" [rounds]
set -e
out=$1; vars=$2; rounds=${3:-2}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
for spec in $vars; do
  name=${spec%%:*}; flags=${spec#*:}
  bash tools/build_variant.sh "$name" ${flags//,/ } > "$out/build_$name.txt" 2>&1
done
for r in $(seq 1 $rounds); do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/prod_table_$r.json" 2>> "$out/err.txt"
  for spec in $vars; do
    name=${spec%%:*}
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$root/leveldb-rs_amd/lib/variants/liblvgpu_$name.so \
      timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/${name}_table_$r.json" 2>> "$out/err.txt"
  done
done
echo table ab done
