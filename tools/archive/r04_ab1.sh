#!/bin/bash
# (Run once in round 4, profiles/r04/ab1/; the switch it measured was then retired with its code.)
# Round 4 A/B pass 1: hash tests + the hash bench (product: XCD-aware sets,
# packed keys with the deferred length shuffle) alternated with the
# round-robin placement (LVK_HASH_XCD_MAP=0); the few-long-buffer bench with
# the hinted offsets call; then the seal sector-merge A/B (tools/r04_seal_ab.sh).
# usage: tools/r04_ab1.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/ab1}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_hash.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$out/pytest_hash.txt" 2>&1 &&
bash tools/build_variant.sh noxcd -DLVK_HASH_XCD_MAP=0 > "$out/build_noxcd.txt" 2>&1 &&
var=$root/leveldb-rs_amd/lib/variants/liblvgpu_noxcd.so &&
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 > "$out/prod_hash_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$var timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 \
    > "$out/noxcd_hash_$r.json" 2>> "$out/err.txt" || exit 1
done &&
echo "hash ab done" &&
timeout -k 10 300 python3 bench.py --long > "$out/long.json" 2> "$out/long.err" &&
echo "long done" &&
bash tools/r04_seal_ab.sh "$out/seal" &&
echo "all steps done"
