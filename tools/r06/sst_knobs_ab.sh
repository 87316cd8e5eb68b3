#!/bin/bash
# Round 6 (final): the table walk's kept knobs re-swept after the seal's
# explicit wait: 4 rows per seal batch (LVK_SEAL_ROWS=4, on the G = 16
# image), runs of 2 or 8 blocks per group (LVK_SST_RUN), against the
# product (3 rows, runs of 4).
set -o pipefail
out=${1:-gpurun_out/r06sk}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
bash tools/build_variant.sh s4 -DLVK_SEAL_ROWS=4 > "$out/build.txt" 2>&1 || exit 1
bash tools/build_variant.sh r2 -DLVK_SST_RUN=2 >> "$out/build.txt" 2>&1 || exit 1
bash tools/build_variant.sh r8 -DLVK_SST_RUN=8 >> "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
for v in s4 r2 r8; do
  LVGPU_SST_STRESS_TRIALS=100 LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_table.py tests/test_gpu_table_stress.py -x -q --timeout 120 --timeout-method thread > "$out/pytest_$v.txt" 2>&1 || exit 1
done
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" || exit 1
  for v in s4 r2 r8; do
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_$v.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/${v}_$r.json" 2>> "$out/err.txt" || exit 1
  done
done
for f in "$out"/prod_*.json "$out"/s4_*.json "$out"/r2_*.json "$out"/r8_*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['seal']['frac_of_8TBps'], d['seal']['ms_avg'], d['verify']['frac_of_8TBps'])" "$f"; done
