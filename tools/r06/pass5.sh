#!/bin/bash
# Round 6: the continuous SST walk with its fast path (every group's blocks
# chained): table GPU tests, then seal / verify against the per-unit walk
# (LVK_SST_STREAM=0), interleaved, and the pipelined-recovery ramp A/B.
set -o pipefail
out=${1:-gpurun_out/r06p5}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_table.py tests/test_gpu_table_stress.py -x -q --timeout 120 --timeout-method thread > "$out/pytest_table.txt" 2>&1 || exit 1
bash tools/build_variant.sh unit -DLVK_SST_STREAM=0 > "$out/build.txt" 2>&1 || exit 1
bash tools/build_variant.sh noramp -DLVK_PIPE_FIRST_MB=32 >> "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/table_prod_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_unit.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/table_unit_$r.json" 2>> "$out/err.txt" || exit 1
done
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 > "$out/wal_prod_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_noramp.so timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 > "$out/wal_noramp_$r.json" 2>> "$out/err.txt" || exit 1
done
echo pass5 done
