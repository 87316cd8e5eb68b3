#!/bin/bash
# Round 5: the WAL framing's sort key from the unit's exact batch count on the
# 256-B row grid (LVK_WAL_KEY_AT=1) against the product, five-launch scan,
# three interleaved reps; then the WAL GPU tests on the variant.
# usage: tools/r05_kat.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05kat}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
bash tools/build_variant.sh kat -DLVK_WAL_KEY_AT=1 > "$out/build.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --wal-device --wal-path 2 --cpu-seconds 0 > "$out/wal_prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_kat.so timeout -k 10 200 python3 bench.py --wal-device --wal-path 2 --cpu-seconds 0 \
    > "$out/wal_kat_$r.json" 2>> "$out/err.txt" || exit 1
done
for f in "$out"/*_*.json; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['roofline']['frac'], d['roofline'].get('ms_avg'))" "$f"; done
LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_kat.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_wal.py tests/test_wal_log.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest_kat.txt" 2>&1 || { tail -30 "$out/pytest_kat.txt"; exit 1; }
tail -2 "$out/pytest_kat.txt"
echo "all steps done"
