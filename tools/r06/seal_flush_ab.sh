#!/bin/bash
# Round 6 (final): the seal flushing its trailers every round or every two
# rounds (LVK_SEAL_FLUSH=1 / 2, a kept tuning knob) against the product's 16
# (one flush per wave at its end).  A trailer written right after its block
# was walked may find the block's tail line still in L2 (the tail granule is
# an L2-allocating load), so the line would be written back whole.
set -o pipefail
out=${1:-gpurun_out/r06fl}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
bash tools/build_variant.sh f1 -DLVK_SEAL_FLUSH=1 > "$out/build.txt" 2>&1 || exit 1
bash tools/build_variant.sh f2 -DLVK_SEAL_FLUSH=2 >> "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
LVGPU_SST_STRESS_TRIALS=200 LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_f1.so timeout -k 10 300 python3 -u -m pytest tests/test_table.py tests/test_gpu_table_stress.py -x -q --timeout 120 --timeout-method thread > "$out/pytest_f1.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" || exit 1
  for v in f1 f2; do
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_$v.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/${v}_$r.json" 2>> "$out/err.txt" || exit 1
  done
done
for f in "$out"/prod_*.json "$out"/f1_*.json "$out"/f2_*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['seal']['frac_of_8TBps'], d['seal']['ms_avg'], d['verify']['frac_of_8TBps'])" "$f"; done
