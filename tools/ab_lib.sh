#!/bin/bash
# A/B of the product library against one experiment variant on the same box:
#   tools/ab_lib.sh OUTDIR VARIANT_NAME -DLVK_FOO=0 ...
# Alternates product / variant twice over C2, C4, C3-offsets, the SST
# trailer bench and the device WAL scan; one JSON line per run in OUTDIR.
set -e
out=$1; name=$2; shift 2
mkdir -p "$out"
bash "$(dirname "$0")/build_variant.sh" "$name" "$@" > "$out/build.txt" 2>&1
var=$GRAFT_REPO_ROOT/leveldb-rs_amd/lib/variants/liblvgpu_$name.so
run() {  # tag, then bench args
  local tag=$1; shift
  timeout -k 10 200 python -u bench.py "$@" > "$out/$tag.json" 2>> "$out/err.txt"
}
for r in 1 2; do
  for w in c2 c4 c3; do
    run "prod_${w}_$r" --workload $w --api offsets --cpu-seconds 0 --traffic off
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$var run "var_${w}_$r" --workload $w --api offsets --cpu-seconds 0 --traffic off
  done
  run "prod_table_$r" --table
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$var run "var_table_$r" --table
  run "prod_wal_$r" --wal-device
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$var run "var_wal_$r" --wal-device
done
echo ab done
