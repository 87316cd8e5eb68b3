#!/bin/bash
# Round 6 (2nd): the seal's wait-count mode under the file-order runs
# (LVK_SEAL_EXACT=2: every load unconditional, as verify runs) against the
# product (masked loads), interleaved, plus the table GPU tests on the variant.
# (The knob lived in commit c6b7f0d only; check that commit out to rerun.)
set -o pipefail
out=${1:-gpurun_out/r06seal}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
bash tools/build_variant.sh exact2 -DLVK_SEAL_EXACT=2 > "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_exact2.so timeout -k 10 300 python3 -u -m pytest tests/test_table.py tests/test_gpu_table_stress.py -x -q --timeout 120 --timeout-method thread > "$out/pytest_exact2.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_exact2.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/exact2_$r.json" 2>> "$out/err.txt" || exit 1
done
for f in "$out"/*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['seal']['frac_of_8TBps'], d['verify']['frac_of_8TBps'])" "$f"; done
