#!/bin/bash
# Round 6 (final): the seal in two launches (LVK_SEAL_SPLIT=1): the walk
# stores each masked CRC by block index, as verify stores its status words,
# and seal_trailers_kernel writes the trailers -- against the product, whose
# walking waves write them at their end (~10 us of ~200, seal_nostore/).
# (Results in profiles/r06/seal_split/; the knob lived in 34e25c4 and was reverted.)
set -o pipefail
out=${1:-gpurun_out/r06split}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
bash tools/build_variant.sh split -DLVK_SEAL_SPLIT=1 > "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
LVGPU_SST_STRESS_TRIALS=400 LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_split.so timeout -k 10 300 python3 -u -m pytest tests/test_table.py tests/test_gpu_table_stress.py -x -q --timeout 120 --timeout-method thread > "$out/pytest_split.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_split.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/split_$r.json" 2>> "$out/err.txt" || exit 1
done
for f in "$out"/prod_*.json "$out"/split_*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['seal']['frac_of_8TBps'], d['seal']['ms_avg'], d['verify']['frac_of_8TBps'])" "$f"; done
