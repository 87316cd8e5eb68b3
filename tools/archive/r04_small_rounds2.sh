#!/bin/bash
# Round 4, after the unsort: the class kernel's small-class wave rule
# (LVK_SMALL_ROUNDS: rounds per small-class wave, product 26) re-measured --
# 52 and 104 -- on C2 / C4 and the WAL scan, alternated.
# usage: tools/r04_small_rounds2.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/small_rounds2}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
for k in 52 104; do bash tools/build_variant.sh sr$k -DLVK_SMALL_ROUNDS=$k >> "$out/build.txt" 2>&1 || exit 1; done
F="--cpu-seconds 0 --traffic off --c5-strong off"
run() { local tag=$1; shift
  timeout -k 10 200 python3 bench.py "$@" > "$out/${tag}_prod_$r.json" 2>> "$out/err.txt" || return 1
  for k in 52 104; do
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_sr$k.so timeout -k 10 200 python3 bench.py "$@" > "$out/${tag}_sr${k}_$r.json" 2>> "$out/err.txt" || return 1
  done; }
for r in 1 2; do
  run c2 --workload c2 --api offsets $F &&
  run c4 --workload c4 --api offsets $F &&
  run wal --wal-device --cpu-seconds 0 || exit 1
done &&
echo "all steps done"
