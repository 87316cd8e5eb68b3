#!/bin/bash
# (Run once in round 4, profiles/r04/new_ab/; the hash switches it measured -- LVK_HASH_DEEP, LVK_HASH_MASKED_META -- were then retired with their code.)
# Round 4: the product with exact wait counts in the sorted walk (class and
# fused kernels) and the two-deep hash, against the previous product
# (variant "old": LVK_WALK_EXACT=0 LVK_HASH_DEEP=0 LVK_HASH_WGS_PER_CU=8).
# The whole GPU suite and smoke on the product, then the affected bench
# lines alternated.  usage: tools/r04_new_ab.sh OUTDIR [rounds]
set -o pipefail
out=${1:-gpurun_out/new_ab}
rounds=${2:-2}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
V=$root/leveldb-rs_amd/lib/variants/liblvgpu_old.so
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest.txt" 2>&1 &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.txt" 2>&1 &&
bash tools/build_variant.sh old -DLVK_WALK_EXACT=0 -DLVK_HASH_DEEP=0 -DLVK_HASH_WGS_PER_CU=8 > "$out/build.txt" 2>&1 || exit 1
F="--cpu-seconds 0 --traffic off --c5-strong off"
run() { local tag=$1; shift
  timeout -k 10 200 python3 bench.py "$@" > "$out/${tag}_prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$V timeout -k 10 200 python3 bench.py "$@" > "$out/${tag}_old_$r.json" 2>> "$out/err.txt"; }
for r in $(seq 1 $rounds); do
  run c3o --workload c3 --api offsets $F &&
  run c2 --workload c2 --api offsets $F &&
  run c4 --workload c4 --api offsets $F &&
  run wal --wal-device --cpu-seconds 0 &&
  run hash --hash --cpu-seconds 0 &&
  run long --long || exit 1
done &&
echo "all steps done"
