#!/bin/bash
# Round 6: the continuous SST walk against the per-unit walk (LVK_SST_STREAM=0)
# on one box: the table GPU tests, then seal / verify interleaved twice.
set -o pipefail
out=${1:-gpurun_out/r06sst_ab}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_table.py tests/test_gpu_table_stress.py -x -q --timeout 120 --timeout-method thread > "$out/pytest_table.txt" 2>&1 || exit 1
bash tools/build_variant.sh unit -DLVK_SST_STREAM=0 > "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/table_prod_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_unit.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/table_unit_$r.json" 2>> "$out/err.txt" || exit 1
done
for f in "$out"/table_*.json; do python3 -c "
import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1].split('/')[-1], d['seal']['frac_of_8TBps'], d['verify']['frac_of_8TBps'])" "$f"; done
