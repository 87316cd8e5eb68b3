#!/bin/bash
# Round 5: pipelined host WAL recovery -- chunk 0 published before chunk 1 is
# copied (product) vs the old order, 3 copy threads, 16 / 64 MiB chunks; the
# --wal line's recovery_pipelined, two interleaved reps.  usage: tools/r05_pipe.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05pipe}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
bash tools/build_variant.sh e0 -DLVK_PIPE_EARLY_FIRST=0 > "$out/build.txt" 2>&1 &&
bash tools/build_variant.sh t3 -DLVK_PIPE_COPY_THREADS=3 >> "$out/build.txt" 2>&1 &&
bash tools/build_variant.sh c16 -DLVK_PIPE_CHUNK_MB=16 >> "$out/build.txt" 2>&1 &&
bash tools/build_variant.sh c64 -DLVK_PIPE_CHUNK_MB=64 >> "$out/build.txt" 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" || exit 1
  for v in e0 t3 c16 c64; do
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_$v.so timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 \
      > "$out/${v}_$r.json" 2>> "$out/err.txt" || exit 1
  done
done
for f in "$out"/*_[12].json; do python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['recovery_pipelined']
print(sys.argv[1], r['GiB_per_s'], r['ms'], r.get('parts_ms'))" "$f"; done
echo "all steps done"
