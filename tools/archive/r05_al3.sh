#!/bin/bash
# Round 5: 3 rows per batch in the class kernel's aligned-row walk
# (LVK_AL_ROWS=3, on the table image's Shift_768) against the product's 4:
# C2 / C4 / C3 via offsets and the five-launch WAL scan, two interleaved reps;
# then the offsets-API and WAL GPU tests on the variant.  usage: tools/r05_al3.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05al3}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
bash tools/build_variant.sh al3 -DLVK_AL_ROWS=3 > "$out/build.txt" 2>&1 || exit 1
LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_al3.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_batch.py tests/test_gpu_wal.py \
  tests/test_gpu_stress.py tests/test_gpu_wal_stress.py -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest_al3.txt" 2>&1 || { tail -30 "$out/pytest_al3.txt"; exit 1; }
tail -1 "$out/pytest_al3.txt"
run() { local tag=$1; shift; timeout -k 10 200 python3 bench.py "$@" --cpu-seconds 0 --c5-strong off > "$out/$tag.json" 2>> "$out/err.txt"; }
V="env LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_al3.so"
for r in 1 2; do
  run c2_prod_$r --workload c2 --api offsets && $V timeout -k 10 200 python3 bench.py --workload c2 --api offsets --cpu-seconds 0 --c5-strong off > "$out/c2_al3_$r.json" 2>> "$out/err.txt" &&
  run c4_prod_$r --workload c4 --api offsets && $V timeout -k 10 200 python3 bench.py --workload c4 --api offsets --cpu-seconds 0 --c5-strong off > "$out/c4_al3_$r.json" 2>> "$out/err.txt" &&
  run c3o_prod_$r --workload c3 --api offsets && $V timeout -k 10 200 python3 bench.py --workload c3 --api offsets --cpu-seconds 0 --c5-strong off > "$out/c3o_al3_$r.json" 2>> "$out/err.txt" &&
  timeout -k 10 200 python3 bench.py --wal-device --wal-path 2 --cpu-seconds 0 > "$out/wal_prod_$r.json" 2>> "$out/err.txt" &&
  $V timeout -k 10 200 python3 bench.py --wal-device --wal-path 2 --cpu-seconds 0 > "$out/wal_al3_$r.json" 2>> "$out/err.txt" || exit 1
done
for f in "$out"/*_[12].json; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['roofline']['frac'])" "$f"; done
echo "all steps done"
