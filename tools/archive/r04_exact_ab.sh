#!/bin/bash
# Round 4: LVK_WALK_EXACT=1 -- the sorted walk issues the same unconditional
# loads in every step (tail and trailer re-read, next round's entries and
# first batch always requested, clamped), so the compiler's wait counts are
# exact and a batch's fold no longer waits for the prefetch behind it.
# GPU tests under the variant, then offsets C3 / C2 / C4, the WAL device scan
# and the SST table line, product and variant alternated.
# usage: tools/r04_exact_ab.sh OUTDIR [rounds]
set -o pipefail
out=${1:-gpurun_out/exact_ab}
rounds=${2:-2}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
V=$root/leveldb-rs_amd/lib/variants/liblvgpu_exact.so
bash tools/build_variant.sh exact -DLVK_WALK_EXACT=1 > "$out/build.txt" 2>&1 &&
LVGPU_EXPERIMENT=1 LVGPU_LIB=$V timeout -k 10 400 python3 -u -m pytest tests/test_gpu_batch.py tests/test_gpu_stress.py \
  tests/test_gpu_wal.py tests/test_table.py -m gpu -x -q --timeout 120 --timeout-method thread > "$out/pytest_exact.txt" 2>&1 || exit 1
F="--cpu-seconds 0 --traffic off --c5-strong off"
run() { local tag=$1; shift
  timeout -k 10 200 python3 bench.py "$@" > "$out/${tag}_prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$V timeout -k 10 200 python3 bench.py "$@" > "$out/${tag}_exact_$r.json" 2>> "$out/err.txt"; }
for r in $(seq 1 $rounds); do
  run c3o --workload c3 --api offsets $F &&
  run c2 --workload c2 --api offsets $F &&
  run c4 --workload c4 --api offsets $F &&
  run wal --wal-device --cpu-seconds 0 &&
  run table --table --cpu-seconds 0 || exit 1
done &&
echo "all steps done"
