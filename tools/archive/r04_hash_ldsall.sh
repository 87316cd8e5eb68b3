#!/bin/bash
# Round 4: the staged hash fast path reading all 17 window dwords unmasked (LVK_HASH_LDS_ALL=1,
# product) against the masked reads (variant la0).  Hash tests, then the hash bench
# alternated.
# usage: tools/r04_hash_ldsall.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/hash_ldsall}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
timeout -k 10 300 python3 -u -m pytest tests/test_hash.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$out/pytest_hash.txt" 2>&1 &&
bash tools/build_variant.sh la0 -DLVK_HASH_LDS_ALL=0 > "$out/build.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_la0.so timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 \
    > "$out/la0_$r.json" 2>> "$out/err.txt" || exit 1
done &&
echo "all steps done"
