#!/bin/bash
# Round 5: the small length classes in index order (LVK_SMALL_INDEX_ORDER=1:
# classes 0 and 1 one sort key each instead of 64 batch-count buckets, so a
# round's buffers are neighbours in the arena) on C2 / C4 (offsets API) and
# the five-launch WAL scan, against the product, two interleaved reps; then the
# offsets-API and WAL GPU tests on the variant.  usage: tools/r05_sio.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05sio}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
bash tools/build_variant.sh sio -DLVK_SMALL_INDEX_ORDER=1 > "$out/build.txt" 2>&1 || exit 1
run() { local tag=$1; shift; timeout -k 10 200 python3 bench.py "$@" --cpu-seconds 0 --c5-strong off > "$out/$tag.json" 2>> "$out/err.txt"; }
for r in 1 2; do
  run c2_prod_$r --workload c2 --api offsets &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_sio.so run c2_sio_$r --workload c2 --api offsets &&
  run c4_prod_$r --workload c4 --api offsets &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_sio.so run c4_sio_$r --workload c4 --api offsets &&
  timeout -k 10 200 python3 bench.py --wal-device --wal-path 2 --cpu-seconds 0 > "$out/wal_prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_sio.so timeout -k 10 200 python3 bench.py --wal-device --wal-path 2 --cpu-seconds 0 \
    > "$out/wal_sio_$r.json" 2>> "$out/err.txt" || exit 1
done
for f in "$out"/*_*.json; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['roofline']['frac'], d['roofline'].get('ms_avg'))" "$f"; done
LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_sio.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_batch.py tests/test_gpu_wal.py \
  tests/test_gpu_stress.py -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest_sio.txt" 2>&1 || { tail -30 "$out/pytest_sio.txt"; exit 1; }
tail -2 "$out/pytest_sio.txt"
echo "all steps done"
