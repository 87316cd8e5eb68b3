#!/bin/bash
# Round 4: the product (exact waits in the class kernel's walk and the SST
# verify walk, class ranges computed in the kernel for hinted identity lists,
# exact hash prefetch) against the session-start build (abtmp/, variant
# "base") on one box: GPU suite + smoke, then every affected line alternated.
# usage: tools/r04_final_ab.sh OUTDIR [rounds]
set -o pipefail
out=${1:-gpurun_out/final_ab}
rounds=${2:-2}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest.txt" 2>&1 &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.txt" 2>&1 &&
(cd abtmp/leveldb-rs_amd && make -j16 lib/liblvgpu.so > "$root/$out/build.txt" 2>&1) && mkdir -p "$VD" &&
cp abtmp/leveldb-rs_amd/lib/liblvgpu.so "$VD/liblvgpu_base.so" || exit 1
F="--cpu-seconds 0 --traffic off --c5-strong off"
run() { local tag=$1; shift
  timeout -k 10 200 python3 bench.py "$@" > "$out/${tag}_prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_base.so timeout -k 10 200 python3 bench.py "$@" > "$out/${tag}_base_$r.json" 2>> "$out/err.txt"; }
for r in $(seq 1 $rounds); do
  run c3 $F &&
  run c3o --workload c3 --api offsets $F &&
  run c2 --workload c2 --api offsets $F &&
  run c4 --workload c4 --api offsets $F &&
  run wal --wal-device --cpu-seconds 0 &&
  run table --table --cpu-seconds 0 &&
  run long --long || exit 1
done &&
echo "all steps done"
