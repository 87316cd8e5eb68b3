#!/bin/bash
# (Run once in round 4, profiles/r04/join_grid/; LVK_JOIN_GRID_N was then retired with its code: no difference.)
# Round 4: combine_long_kernel launched with min(buffers, CUs) workgroups
# (product) against one per CU (variant g0), on the few-long-buffer calls;
# the GPU batch tests under the product first.  usage: tools/r04_join_grid.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/join_grid}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_batch.py tests/test_gpu_stress.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > "$out/pytest.txt" 2>&1 &&
bash tools/build_variant.sh g0 -DLVK_JOIN_GRID_N=0 > "$out/build.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --long > "$out/long_prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_g0.so timeout -k 10 200 python3 bench.py --long > "$out/long_g0_$r.json" 2>> "$out/err.txt" || exit 1
done &&
echo "all steps done"
