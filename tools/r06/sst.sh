#!/bin/bash
# Round 6: SST file-order runs (LVK_SST_RUN).  The table
# GPU tests, then bench.py --table for the product (k = 4) against variants
# k = 1 (round 5's order), 2 and 8, interleaved twice, then FETCH/WRITE per
# kernel and kernel stats for the product (tools/prof_8f.sh table).
set -o pipefail
out=${1:-gpurun_out/r06sst}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_table.py tests/test_gpu_table_stress.py tests/test_gpu_batch.py -k "table or sst or seal or verify" -x -q --timeout 120 --timeout-method thread > "$out/pytest_table.txt" 2>&1 || exit 1
for k in 1 2 8; do bash tools/build_variant.sh run$k -DLVK_SST_RUN=$k >> "$out/build.txt" 2>&1 || exit 1; done
VD=$root/leveldb-rs_amd/lib/variants
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" || exit 1
  for k in 1 2 8; do
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_run$k.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/run${k}_$r.json" 2>> "$out/err.txt" || exit 1
  done
done
bash tools/prof_8f.sh "$out/prof" table > "$out/prof.log" 2>&1 || exit 1
echo done
