#!/bin/bash
# Product vs several experiment variants on the offsets workloads, alternated:
#   tools/ab_multi.sh OUT "name1:-DFOO=1 name2:-DFOO=2" "c2 c4" [rounds]
set -e
out=$1; vars=$2; works=$3; rounds=${4:-2}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
for spec in $vars; do
  name=${spec%%:*}; flags=${spec#*:}
  bash tools/build_variant.sh "$name" ${flags//,/ } > "$out/build_$name.txt" 2>&1
done
for r in $(seq 1 $rounds); do
  for w in $works; do
    timeout -k 10 200 python3 bench.py --workload $w --api offsets --cpu-seconds 0 --traffic off > "$out/prod_${w}_$r.json" 2>> "$out/err.txt"
    for spec in $vars; do
      name=${spec%%:*}
      LVGPU_EXPERIMENT=1 LVGPU_LIB=$root/leveldb-rs_amd/lib/variants/liblvgpu_$name.so \
        timeout -k 10 200 python3 bench.py --workload $w --api offsets --cpu-seconds 0 --traffic off > "$out/${name}_${w}_$r.json" 2>> "$out/err.txt"
    done
  done
done
echo multi ab done
