#!/bin/bash
# Round 4: the sorted path writes each CRC at its sorted position and the
# join launch unsorts them (out[i] = tmp[pos[i]], whole lines in buffer
# order) instead of the class kernel's scattered single-word stores.  The
# GPU suite and smoke on the product, then C2 / C4 / C3 via offsets / the
# WAL scan / the few-long-buffer calls against the session-start build
# (abtmp/, variant "base"), alternated.  usage: tools/r04_unsort_ab.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/unsort_ab}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest.txt" 2>&1 &&
LVGPU_STRESS_TRIALS=120 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_stress.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > "$out/stress120.txt" 2>&1 &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.txt" 2>&1 &&
(cd abtmp/leveldb-rs_amd && make -j16 lib/liblvgpu.so > "$root/$out/build.txt" 2>&1) && mkdir -p "$VD" &&
cp abtmp/leveldb-rs_amd/lib/liblvgpu.so "$VD/liblvgpu_base.so" || exit 1
F="--cpu-seconds 0 --traffic off --c5-strong off"
run() { local tag=$1; shift
  timeout -k 10 200 python3 bench.py "$@" > "$out/${tag}_prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_base.so timeout -k 10 200 python3 bench.py "$@" > "$out/${tag}_base_$r.json" 2>> "$out/err.txt"; }
for r in 1 2; do
  run c2 --workload c2 --api offsets $F &&
  run c4 --workload c4 --api offsets $F &&
  run c3o --workload c3 --api offsets $F &&
  run long --long || exit 1
done &&
timeout -k 10 300 python3 bench.py --workload c2 --api offsets --cpu-seconds 5 > "$out/c2_parity.json" 2>> "$out/err.txt" &&
echo "all steps done"
