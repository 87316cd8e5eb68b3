#!/bin/bash
# Round 4, after the verify walk's exact waits: rows per batch of the table
# walk (LVK_SST_ROWS, product 3) re-measured at 4 (the walk allows 3 or 4), bench --table
# alternated.  usage: tools/r04_sst_rows.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/sst_rows}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
for k in 4; do bash tools/build_variant.sh rows$k -DLVK_SST_ROWS=$k >> "$out/build.txt" 2>&1 || exit 1; done
LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_rows4.so timeout -k 10 300 python3 -u -m pytest tests/test_table.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > "$out/pytest_rows4.txt" 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/table_prod_$r.json" 2>> "$out/err.txt" || exit 1
  for k in 4; do
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_rows$k.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 \
      > "$out/table_rows${k}_$r.json" 2>> "$out/err.txt" || exit 1
  done
done &&
echo "all steps done"
