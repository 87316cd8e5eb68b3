#!/bin/bash
# Round 4: sorted-walk wait-count mode 2 (unconditional loads within each
# path, no per-step re-reads) for the table walk (t2), the class kernel's
# lists (w2) and the fused small-batch kernel (f2), each against the product
# (class lists mode 1, table and fused mode 0).  GPU tests of the touched
# files under each variant, then the bench lines alternated.
# usage: tools/r04_mode2_ab.sh OUTDIR [rounds]
set -o pipefail
out=${1:-gpurun_out/mode2_ab}
rounds=${2:-2}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
bash tools/build_variant.sh t2 -DLVK_TABLE_EXACT=2 > "$out/build.txt" 2>&1 &&
bash tools/build_variant.sh w2 -DLVK_WALK_EXACT=2 >> "$out/build.txt" 2>&1 &&
bash tools/build_variant.sh f2 -DLVK_FUSED_EXACT=2 >> "$out/build.txt" 2>&1 || exit 1
for v in t2 w2 f2; do
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_$v.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_batch.py \
    tests/test_gpu_stress.py tests/test_gpu_wal.py tests/test_table.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$out/pytest_$v.txt" 2>&1 || exit 1
done
F="--cpu-seconds 0 --traffic off --c5-strong off"
run() { local tag=$1 v=$2; shift 2
  timeout -k 10 200 python3 bench.py "$@" > "$out/${tag}_prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_$v.so timeout -k 10 200 python3 bench.py "$@" > "$out/${tag}_${v}_$r.json" 2>> "$out/err.txt"; }
for r in $(seq 1 $rounds); do
  run table t2 --table --cpu-seconds 0 &&
  run c3o w2 --workload c3 --api offsets $F &&
  run c2 w2 --workload c2 --api offsets $F &&
  run c4 w2 --workload c4 --api offsets $F &&
  run wal w2 --wal-device --cpu-seconds 0 &&
  run long f2 --long || exit 1
done &&
echo "all steps done"
