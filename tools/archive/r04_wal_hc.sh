#!/bin/bash
# (Run once in round 4, profiles/r04/wal_hc/; LVK_WAL_HC_COOP was then retired with its code: slower.)
# Round 4: wal_hist writing its header cache block by block with consecutive
# lanes (LVK_WAL_HC_COOP=1) against every lane storing its own block's
# headers (variant hc0).  WAL GPU tests, then bench --wal-device alternated.
# usage: tools/r04_wal_hc.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/wal_hc}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_wal.py tests/test_wal_log.py tests/test_wal_boundary.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > "$out/pytest.txt" 2>&1 &&
bash tools/build_variant.sh hc0 -DLVK_WAL_HC_COOP=0 > "$out/build.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --wal-device --cpu-seconds 0 > "$out/wal_prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_hc0.so timeout -k 10 200 python3 bench.py --wal-device --cpu-seconds 0 \
    > "$out/wal_hc0_$r.json" 2>> "$out/err.txt" || exit 1
done &&
echo "all steps done"
