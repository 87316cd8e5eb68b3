#!/bin/bash
# Round 6 (final), timing study: the seal writing whole 32-B / 64-B sectors
# around each trailer (LVK_SEAL_SECTOR=32/64: re-read, patched, written back;
# valid only when no two trailers share a sector, as in bench.py's table)
# against the product's 5-B partial writes.
# (Results in profiles/r06/seal_sector/; the knobs lived in 02e8055 and were reverted.)
set -o pipefail
out=${1:-gpurun_out/r06sec}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
bash tools/build_variant.sh s32 -DLVK_SEAL_SECTOR=32 > "$out/build32.txt" 2>&1 || exit 1
bash tools/build_variant.sh s64 -DLVK_SEAL_SECTOR=64 > "$out/build64.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_s32.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/s32_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_s64.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/s64_$r.json" 2>> "$out/err.txt" || exit 1
done
for f in "$out"/prod_*.json "$out"/s32_*.json "$out"/s64_*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['seal']['frac_of_8TBps'], d['seal']['ms_avg'], d['verify']['frac_of_8TBps'])" "$f"; done
