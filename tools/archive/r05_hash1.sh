#!/bin/bash
# Round 5: the hash with two keys per lane (LVK_HASH_KPL=2; k2a: 4,864-B
# stages at 8 workgroups per CU, k2b: 6,144-B stages at 6) against the
# product, the variants' hash tests first; then the --wal host line (the
# pipelined recovery pass and its parts).  usage: tools/r05_hash1.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05h}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
bash tools/build_variant.sh k2a -DLVK_HASH_KPL=2 > "$out/build.txt" 2>&1 &&
bash tools/build_variant.sh k2b -DLVK_HASH_KPL=2 -DLVK_HASH_SPAN2=6144 -DLVK_HASH_WGS_PER_CU=6 >> "$out/build.txt" 2>&1 || exit 1
for v in k2a k2b; do
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_hash.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > "$out/pytest_$v.txt" 2>&1 || exit 1
done
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_k2a.so timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 \
    > "$out/k2a_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_k2b.so timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 \
    > "$out/k2b_$r.json" 2>> "$out/err.txt" || exit 1
done &&
timeout -k 10 600 python3 bench.py --wal --cpu-seconds 0 > "$out/wal_host.json" 2> "$out/wal_host.err" &&
echo "all steps done"
