#!/bin/bash
# Round 4: the hash chain without the tail-word capture (LVK_HASH_TAIL_READ=1,
# product: the tail's dwords re-read after the chain) against the capture in
# the loop (variant tr0).  Hash tests, then the hash bench alternated.
# usage: tools/r04_hash_tail.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/hash_tail}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
timeout -k 10 300 python3 -u -m pytest tests/test_hash.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$out/pytest_hash.txt" 2>&1 &&
bash tools/build_variant.sh tr0 -DLVK_HASH_TAIL_READ=0 > "$out/build.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_tr0.so timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 \
    > "$out/tr0_$r.json" 2>> "$out/err.txt" || exit 1
done &&
echo "all steps done"
