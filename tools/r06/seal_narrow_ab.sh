#!/bin/bash
# Round 6 (final): the seal flush with no load (LVK_SEAL_NARROW=1: the trailer
# offset and type byte staged in LDS; the product re-reads the handle and type)
# against the product.
# (Measured flat, profiles/r06/seal_narrow/; the knob lived in 6564f5b and was reverted.)
set -o pipefail
out=${1:-gpurun_out/r06nw}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
bash tools/build_variant.sh nw -DLVK_SEAL_NARROW=1 > "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
LVGPU_SST_STRESS_TRIALS=400 LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_nw.so timeout -k 10 300 python3 -u -m pytest tests/test_table.py tests/test_gpu_table_stress.py -x -q --timeout 120 --timeout-method thread > "$out/pytest_nw.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_nw.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/nw_$r.json" 2>> "$out/err.txt" || exit 1
done
for f in "$out"/prod_*.json "$out"/nw_*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['seal']['frac_of_8TBps'], d['verify']['frac_of_8TBps'])" "$f"; done
