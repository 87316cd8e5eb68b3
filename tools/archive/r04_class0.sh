#!/bin/bash
# (Run once in round 4, profiles/r04/class0/; LVK_CLASS0_G4 was not kept: WAL 0.633 -> 0.573, C2 unchanged.)
# Round 4: class 0 (units <= 256 B) walked by 4-lane groups (variant c0g4:
# LVK_CLASS0_G4=1) against one lane per unit (product).  GPU batch tests under
# the variant, then the class-split probe and C2 / C4 / the WAL scan alternated.
# usage: tools/r04_class0.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/class0}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
bash tools/build_variant.sh c0g4 -DLVK_CLASS0_G4=1 > "$out/build.txt" 2>&1 &&
LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_c0g4.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_batch.py \
  tests/test_gpu_stress.py tests/test_gpu_wal.py -m gpu -x -q --timeout 120 --timeout-method thread > "$out/pytest_c0g4.txt" 2>&1 || exit 1
F="--cpu-seconds 0 --traffic off --c5-strong off"
run() { local tag=$1; shift
  timeout -k 10 200 python3 bench.py "$@" > "$out/${tag}_prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_c0g4.so timeout -k 10 200 python3 bench.py "$@" > "$out/${tag}_c0g4_$r.json" 2>> "$out/err.txt"; }
for r in 1 2; do
  run c2 --workload c2 --api offsets $F &&
  run c4 --workload c4 --api offsets $F &&
  run wal --wal-device --cpu-seconds 0 || exit 1
done &&
timeout -k 10 200 python3 tools/class_split_probe.py c2 > "$out/split_prod.txt" 2>&1 &&
LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_c0g4.so timeout -k 10 200 python3 tools/class_split_probe.py c2 > "$out/split_c0g4.txt" 2>&1 &&
echo "all steps done"
