#!/bin/bash
# Round 4: wal_hist's touch point (LVK_WAL_TOUCH_HOPS: after how many header
# hops a long chain's remaining lines are touched into L2) -- product 16
# against 8, 12 and 24, bench --wal-device alternated.
# usage: tools/r04_wal_touch.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/wal_touch}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
for h in 8 12 24; do bash tools/build_variant.sh th$h -DLVK_WAL_TOUCH_HOPS=$h >> "$out/build.txt" 2>&1 || exit 1; done
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --wal-device --cpu-seconds 0 > "$out/wal_prod_$r.json" 2>> "$out/err.txt" || exit 1
  for h in 8 12 24; do
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_th$h.so timeout -k 10 200 python3 bench.py --wal-device --cpu-seconds 0 \
      > "$out/wal_th${h}_$r.json" 2>> "$out/err.txt" || exit 1
  done
done &&
echo "all steps done"
