#!/bin/bash
# Round 6 (2nd): the table walk with the next batch's addresses computed a
# step ahead (LVK_WALK_PREADDR=1), so each step issues its loads before any
# address arithmetic (the compiler waited vmcnt(0) at the top of every step
# for registers the arithmetic reused), against the product, interleaved.
out=${1:-gpurun_out/r06pa}
# (The knob lived in commits 3dac183 and e3921bf only; check e3921bf out to rerun.)
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
bash tools/build_variant.sh pa -DLVK_WALK_PREADDR=1 > "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
LVGPU_SST_STRESS_TRIALS=400 LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_pa.so timeout -k 10 300 python3 -u -m pytest tests/test_table.py tests/test_gpu_table_stress.py -x -q --timeout 120 --timeout-method thread > "$out/pytest_pa.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_pa.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/pa_$r.json" 2>> "$out/err.txt" || exit 1
done
for f in "$out"/prod_*.json "$out"/pa_*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['seal']['frac_of_8TBps'], d['verify']['frac_of_8TBps'])" "$f"; done
