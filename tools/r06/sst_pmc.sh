#!/bin/bash
# Round 6: SQ counters of the SST kernels -- the continuous walk (product) and
# the per-unit walk (LVK_SST_STREAM=0) -- one small counter set per pass.
set -o pipefail
out=${1:-gpurun_out/r06sst_pmc}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
bash tools/build_variant.sh unit -DLVK_SST_STREAM=0 > "$out/build.txt" 2>&1 || exit 1
bash tools/pmc_passes.sh "$out/prod" --table > "$out/prod.log" 2>&1 || exit 1
LVGPU_EXPERIMENT=1 LVGPU_LIB=$root/leveldb-rs_amd/lib/variants/liblvgpu_unit.so bash tools/pmc_passes.sh "$out/unit" --table > "$out/unit.log" 2>&1 || exit 1
echo done
