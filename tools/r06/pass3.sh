#!/bin/bash
# Round 6, third GPU pass: the whole GPU suite after the knob cleanup and the
# new tests, then the pipelined recovery with the chunk ramp (product,
# LVK_PIPE_FIRST_MB=2) against no ramp (variant, 32), interleaved 3 times.
set -o pipefail
out=${1:-gpurun_out/r06p3}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/pytest_gpu.txt" 2>&1 || exit 1
bash tools/build_variant.sh noramp -DLVK_PIPE_FIRST_MB=32 > "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 > "$out/wal_prod_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_noramp.so timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 > "$out/wal_noramp_$r.json" 2>> "$out/err.txt" || exit 1
done
bash tools/build_variant.sh rows2 -DLVK_SST_ROWS=2 >> "$out/build.txt" 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/table_prod_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_rows2.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/table_rows2_$r.json" 2>> "$out/err.txt" || exit 1
done
echo pass3 done
