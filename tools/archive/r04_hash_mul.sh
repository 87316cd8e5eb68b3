#!/bin/bash
# Round 4 timing probe: is the hash chain's 32-bit multiply (v_mul_lo_u32)
# its bound?  Variant m24 (LVK_EXP_HASH_MUL24, wrong hashes) multiplies with
# v_mul_u32_u24; bench --hash without parity, alternated with the product.
# usage: tools/r04_hash_mul.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/hash_mul}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
bash tools/build_variant.sh m24 -DLVK_EXP_HASH_MUL24=1 > "$out/build.txt" 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_m24.so timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 \
    > "$out/m24_$r.json" 2>> "$out/err.txt" || exit 1
done &&
echo "all steps done"
