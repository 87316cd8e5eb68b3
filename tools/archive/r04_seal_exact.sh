#!/bin/bash
# (Run once in round 4, profiles/r04/seal_exact/; LVK_SEAL_EXACT was then retired with its code: slower.)
# Round 4: the SST seal walk with exact wait counts and unconditional trailer
# stores (variant se2: LVK_SEAL_EXACT=2) against the product (masked loads and
# stores).  Table GPU tests under the variant, then bench --table alternated.
# usage: tools/r04_seal_exact.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/seal_exact}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
bash tools/build_variant.sh se2 -DLVK_SEAL_EXACT=2 > "$out/build.txt" 2>&1 &&
LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_se2.so timeout -k 10 300 python3 -u -m pytest tests/test_table.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > "$out/pytest_se2.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/table_prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_se2.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 \
    > "$out/table_se2_$r.json" 2>> "$out/err.txt" || exit 1
done &&
echo "all steps done"
