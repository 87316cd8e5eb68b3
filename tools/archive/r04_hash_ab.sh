#!/bin/bash
# (Run once in round 4, profiles/r04/hash_ab/; the switch it measured was then retired with its code.)
# Round 4: the branch-free hash chain and span staging (LVK_HASH_BRANCHFREE=1,
# the product) against the round-3 branchy form (=0): hash tests, then the
# hash bench alternated three times.  usage: tools/r04_hash_ab.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/hash_ab}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_hash.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$out/pytest_hash.txt" 2>&1 &&
bash tools/build_variant.sh branchy -DLVK_HASH_BRANCHFREE=0 > "$out/build.txt" 2>&1 &&
var=$root/leveldb-rs_amd/lib/variants/liblvgpu_branchy.so &&
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 > "$out/prod_hash_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$var timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 \
    > "$out/branchy_hash_$r.json" 2>> "$out/err.txt" || exit 1
done &&
echo "all steps done"
