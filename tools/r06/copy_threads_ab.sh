#!/bin/bash
# Round 6 (2nd): the pipelined scan's staging-copy threads (LVK_PIPE_COPY_THREADS,
# product 4) with the bench process on the GPU's socket (bench --wal default
# placement): 4 / 6 / 8, interleaved, three reps.
set -o pipefail
out=${1:-gpurun_out/r06ct}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
bash tools/build_variant.sh ct6 -DLVK_PIPE_COPY_THREADS=6 > "$out/build.txt" 2>&1 || exit 1
bash tools/build_variant.sh ct8 -DLVK_PIPE_COPY_THREADS=8 >> "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 > "$out/ct4_$r.json" 2>> "$out/err.txt" || exit 1
  for v in 6 8; do
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_ct$v.so timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 > "$out/ct${v}_$r.json" 2>> "$out/err.txt" || exit 1
  done
done
for f in "$out"/ct*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['recovery_pipelined']['GiB_per_s'], d['recovery_pipelined_pinned_log']['GiB_per_s'], d['recovery_pipelined']['parts_ms'])" "$f"; done
