#!/bin/bash
# (Run once in round 4, profiles/r04/hash_glds/; the switch it measured was then retired with its code.)
# Round 4: the LDS-DMA hash kernel (LVK_HASH_GLDS=1: the next set's span
# prefetched into a second LDS stage) -- parity under the hash tests, then the
# hash bench alternated with the product library.  usage: tools/r04_hash_glds_ab.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/hash_glds}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
bash tools/build_variant.sh glds -DLVK_HASH_GLDS=1 > "$out/build.txt" 2>&1 &&
var=$root/leveldb-rs_amd/lib/variants/liblvgpu_glds.so &&
LVGPU_EXPERIMENT=1 LVGPU_LIB=$var timeout -k 10 300 python3 -u -m pytest tests/test_hash.py -m gpu -x -v \
  --timeout 120 --timeout-method thread > "$out/pytest_hash_glds.txt" 2>&1 &&
echo "variant parity ok" &&
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 > "$out/prod_hash_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$var timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 \
    > "$out/glds_hash_$r.json" 2>> "$out/err.txt" || exit 1
done &&
echo "all steps done"
