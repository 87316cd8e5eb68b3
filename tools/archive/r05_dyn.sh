#!/bin/bash
# Round 5: the class kernel's chunked device rounds (LVK_CLASS_DYN=1: the
# large rounds from one device counter in chunks of 16 instead of b + k*grid
# per workgroup) on C2 / C4 (offsets API) and the five-launch WAL scan,
# against the product, two interleaved reps.  usage: tools/r05_dyn.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05dyn}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
bash tools/build_variant.sh dyn -DLVK_CLASS_DYN=1 > "$out/build.txt" 2>&1 || exit 1
run() { local tag=$1; shift; timeout -k 10 200 python3 bench.py "$@" --cpu-seconds 0 --c5-strong off > "$out/$tag.json" 2>> "$out/err.txt"; }
for r in 1 2; do
  run c2_prod_$r --workload c2 --api offsets &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_dyn.so run c2_dyn_$r --workload c2 --api offsets &&
  run c4_prod_$r --workload c4 --api offsets &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_dyn.so run c4_dyn_$r --workload c4 --api offsets &&
  timeout -k 10 200 python3 bench.py --wal-device --wal-path 2 --cpu-seconds 0 > "$out/wal_prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_dyn.so timeout -k 10 200 python3 bench.py --wal-device --wal-path 2 --cpu-seconds 0 \
    > "$out/wal_dyn_$r.json" 2>> "$out/err.txt" || exit 1
done
for f in "$out"/*_*.json; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['roofline']['frac'], d['roofline'].get('ms_avg'))" "$f"; done
echo "all steps done"
