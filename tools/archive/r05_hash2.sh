#!/bin/bash
# Round 5: the hash with the next set's span prefetched by LDS-DMA in issue
# order (variant g2: LVK_HASH_GLDS2, 7 workgroups per CU) against the product,
# its hash tests first; then the WAL one-launch scan's per-wave timeline.
# usage: tools/r05_hash2.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05g}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
bash tools/build_variant.sh g2 -DLVK_HASH_GLDS2=1 -DLVK_HASH_WGS_PER_CU=7 > "$out/build.txt" 2>&1 &&
LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_g2.so timeout -k 10 300 python3 -u -m pytest tests/test_hash.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > "$out/pytest_g2.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_g2.so timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 \
    > "$out/g2_$r.json" 2>> "$out/err.txt" || exit 1
done &&
true &&
echo "all steps done"
