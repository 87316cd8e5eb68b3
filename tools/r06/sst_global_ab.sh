#!/bin/bash
# Round 6 (final): the table walk with its trailer loads (verify) and stores
# (seal) in the global address space (LVK_SST_GLOBAL=1) against the product,
# whose flat ones count in lgkmcnt as well as vmcnt.
# (Measured flat, profiles/r06/sst_global/; the knob lived in 3ec5f0f and was reverted.)
set -o pipefail
out=${1:-gpurun_out/r06gl}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
bash tools/build_variant.sh gl -DLVK_SST_GLOBAL=1 > "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
LVGPU_SST_STRESS_TRIALS=400 LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_gl.so timeout -k 10 300 python3 -u -m pytest tests/test_table.py tests/test_gpu_table_stress.py -x -q --timeout 120 --timeout-method thread > "$out/pytest_gl.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_gl.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/gl_$r.json" 2>> "$out/err.txt" || exit 1
done
for f in "$out"/prod_*.json "$out"/gl_*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['seal']['frac_of_8TBps'], d['verify']['frac_of_8TBps'])" "$f"; done
