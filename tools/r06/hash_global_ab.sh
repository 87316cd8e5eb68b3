#!/bin/bash
# Round 6 (final): the hash kernel's direct key loads in the global address
# space (LVK_HASH_GLOBAL=1) against the product, where the compiler merged the
# tail-word loads of the staged (LDS) and direct paths into one flat load.
# (Measured flat, profiles/r06/hash_global/; the knob lived in 3ec5f0f and was reverted.)
set -o pipefail
out=${1:-gpurun_out/r06hg}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
bash tools/build_variant.sh hg -DLVK_HASH_GLOBAL=1 > "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_hg.so timeout -k 10 300 python3 -u -m pytest tests/test_hash.py tests/test_gpu_hash_stress.py -x -q --timeout 120 --timeout-method thread > "$out/pytest_hg.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 --traffic off > "$out/prod_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_hg.so timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 --traffic off > "$out/hg_$r.json" 2>> "$out/err.txt" || exit 1
done
for f in "$out"/prod_*.json "$out"/hg_*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['roofline_hbm']['frac'], d['packed_u64']['roofline_hbm']['frac'], d['packed_u32']['roofline_hbm']['frac'])" "$f"; done
