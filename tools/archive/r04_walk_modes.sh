#!/bin/bash
# Round 4: the class kernel's wait-count mode (LVK_WALK_EXACT 0 / 1 / 2) on
# the offsets C3 / C2 / C4 lines and the WAL device scan, product (mode 1)
# and variants w0, w2 alternated.  usage: tools/r04_walk_modes.sh OUTDIR [rounds]
set -o pipefail
out=${1:-gpurun_out/walk_modes}
rounds=${2:-2}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
bash tools/build_variant.sh w0 -DLVK_WALK_EXACT=0 > "$out/build.txt" 2>&1 &&
bash tools/build_variant.sh w2 -DLVK_WALK_EXACT=2 >> "$out/build.txt" 2>&1 || exit 1
F="--cpu-seconds 0 --traffic off --c5-strong off"
run() { local tag=$1; shift
  timeout -k 10 200 python3 bench.py "$@" > "$out/${tag}_prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_w0.so timeout -k 10 200 python3 bench.py "$@" > "$out/${tag}_w0_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_w2.so timeout -k 10 200 python3 bench.py "$@" > "$out/${tag}_w2_$r.json" 2>> "$out/err.txt"; }
for r in $(seq 1 $rounds); do
  run c3o --workload c3 --api offsets $F &&
  run c2 --workload c2 --api offsets $F &&
  run c4 --workload c4 --api offsets $F &&
  run wal --wal-device --cpu-seconds 0 || exit 1
done &&
echo "all steps done"
