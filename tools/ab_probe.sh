#!/bin/bash
# tools/ab_probe.sh OUT NAME "FLAGS" SCRIPT ARGS... : product vs one variant,
# alternated 3 times, for a probe script that prints one line per run.
set -e
out=$1; name=$2; flags=$3; shift 3
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/build_variant.sh "$name" ${flags//,/ } > "$out/build_$name.txt" 2>&1
for r in 1 2 3; do
  echo "prod $(timeout -k 10 120 python3 "$@" 2>/dev/null | tail -1)" >> "$out/ab.txt"
  echo "$name $(LVGPU_EXPERIMENT=1 LVGPU_LIB=$root/leveldb-rs_amd/lib/variants/liblvgpu_$name.so timeout -k 10 120 python3 "$@" 2>/dev/null | tail -1)" >> "$out/ab.txt"
done
cat "$out/ab.txt"
