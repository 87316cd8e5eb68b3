#!/bin/bash
# Round 5: the pipelined host WAL recovery pass at other chunk sizes and
# staging-copy thread counts (variants), bench.py --wal each.
# usage: tools/r05_walhost.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05wh}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
bash tools/build_variant.sh c8 -DLVK_PIPE_CHUNK_MB=8 > "$out/build.txt" 2>&1 &&
bash tools/build_variant.sh c16 -DLVK_PIPE_CHUNK_MB=16 >> "$out/build.txt" 2>&1 &&
bash tools/build_variant.sh c8t4 -DLVK_PIPE_CHUNK_MB=8 -DLVK_MEMCPY_THREADS=4 >> "$out/build.txt" 2>&1 &&
bash tools/build_variant.sh c32t4 -DLVK_MEMCPY_THREADS=4 >> "$out/build.txt" 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 > "$out/prod.json" 2>> "$out/err.txt" || exit 1
for v in c8 c16 c8t4 c32t4; do
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_$v.so timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 \
    > "$out/$v.json" 2>> "$out/err.txt" || exit 1
done &&
echo "all steps done"
