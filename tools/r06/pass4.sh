#!/bin/bash
# Round 6, fourth GPU pass: the whole GPU suite (continuous SST walk, knob
# cleanup, teardown test), then A/B on one box: the SST trailers with the
# continuous walk (product) against the per-unit walk (LVK_SST_STREAM=0) and
# its 2-row batches (LVK_SST_STREAM=0 LVK_SST_ROWS=2), FETCH/WRITE of the new
# kernel; the pipelined recovery with the chunk ramp (product) against none
# (LVK_PIPE_FIRST_MB=32), interleaved.
set -o pipefail
out=${1:-gpurun_out/r06p4}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/pytest_gpu.txt" 2>&1 || exit 1
bash tools/build_variant.sh unit -DLVK_SST_STREAM=0 > "$out/build.txt" 2>&1 || exit 1
bash tools/build_variant.sh unit2 -DLVK_SST_STREAM=0 -DLVK_SST_ROWS=2 >> "$out/build.txt" 2>&1 || exit 1
bash tools/build_variant.sh noramp -DLVK_PIPE_FIRST_MB=32 >> "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/table_prod_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_unit.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/table_unit_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_unit2.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/table_unit2_$r.json" 2>> "$out/err.txt" || exit 1
done
bash tools/prof_8f.sh "$out/prof" table > "$out/prof.log" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 > "$out/wal_prod_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_noramp.so timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 > "$out/wal_noramp_$r.json" 2>> "$out/err.txt" || exit 1
done
echo pass4 done
