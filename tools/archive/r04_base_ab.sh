#!/bin/bash
# Round 4: is a box slow, or the code?  Builds the session-start tree
# (abtmp/, git archive b0ed367) on the box as variant "base" and runs the
# headline and the latency-sensitive lines against the product, alternated.
# usage: tools/r04_base_ab.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/base_ab}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
(cd abtmp/leveldb-rs_amd && make -j16 lib/liblvgpu.so > "$root/$out/build.txt" 2>&1) && mkdir -p "$VD" &&
cp abtmp/leveldb-rs_amd/lib/liblvgpu.so "$VD/liblvgpu_base.so" || exit 1
F="--cpu-seconds 0 --traffic off --c5-strong off"
run() { local tag=$1; shift
  timeout -k 10 200 python3 bench.py "$@" > "$out/${tag}_prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_base.so timeout -k 10 200 python3 bench.py "$@" > "$out/${tag}_base_$r.json" 2>> "$out/err.txt"; }
for r in 1 2; do
  run c3 $F &&
  run c3o --workload c3 --api offsets $F &&
  run wal --wal-device --cpu-seconds 0 &&
  run hash --hash --cpu-seconds 0 || exit 1
done &&
echo "all steps done"
