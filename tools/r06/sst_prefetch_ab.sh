#!/bin/bash
# Round 6 (final): the table walk requesting its first batches while the
# table image is staged (LVK_SST_PREFETCH=1; wave w touches the first batch of
# its workgroup's w-th first claim) against the product.
# (Results in profiles/r06/sst_prefetch/; the knob lived in 3a6d0fc and was reverted.)
set -o pipefail
out=${1:-gpurun_out/r06pf}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
bash tools/build_variant.sh pf -DLVK_SST_PREFETCH=1 > "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
LVGPU_SST_STRESS_TRIALS=400 LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_pf.so timeout -k 10 300 python3 -u -m pytest tests/test_table.py tests/test_gpu_table_stress.py -x -q --timeout 120 --timeout-method thread > "$out/pytest_pf.txt" 2>&1 || exit 1
for r in ${REPS:-1 2 3 4}; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_pf.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/pf_$r.json" 2>> "$out/err.txt" || exit 1
done
for f in "$out"/prod_*.json "$out"/pf_*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['seal']['frac_of_8TBps'], d['verify']['frac_of_8TBps'])" "$f"; done
