#!/bin/bash
# (Run once in round 4, profiles/r04/hash_wait/; the hash switches it measured -- LVK_HASH_DEEP, LVK_HASH_MASKED_META -- were then retired with their code.)
# Round 4: hash metadata loads and the compiler's wait counts.  prod = every
# metadata load issued by every lane (clamped) with a clean wait state at the
# loop head; masked = the earlier form (exec-masked loads, the prefetch under
# `more`: its first wait per set was a vmcnt(0) covering the prefetch just
# issued); deep6 / deep8 = two sets deep (next set's span in registers), 6 or 8
# workgroups per CU.  Hash tests on prod, then the hash bench alternated.
# usage: tools/r04_hash_wait.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/hash_wait}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
V=$root/leveldb-rs_amd/lib/variants
timeout -k 10 300 python3 -u -m pytest tests/test_hash.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$out/pytest_hash.txt" 2>&1 &&
bash tools/build_variant.sh masked -DLVK_HASH_MASKED_META=1 > "$out/build.txt" 2>&1 &&
bash tools/build_variant.sh deep6 -DLVK_HASH_DEEP=1 -DLVK_HASH_WGS_PER_CU=6 >> "$out/build.txt" 2>&1 &&
bash tools/build_variant.sh deep8 -DLVK_HASH_DEEP=1 >> "$out/build.txt" 2>&1 &&
LVGPU_EXPERIMENT=1 LVGPU_LIB=$V/liblvgpu_deep6.so timeout -k 10 300 python3 -u -m pytest tests/test_hash.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > "$out/pytest_hash_deep6.txt" 2>&1 &&
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$V/liblvgpu_masked.so timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 \
    > "$out/masked_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$V/liblvgpu_deep6.so timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 \
    > "$out/deep6_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$V/liblvgpu_deep8.so timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 \
    > "$out/deep8_$r.json" 2>> "$out/err.txt" || exit 1
done &&
echo "all steps done"
