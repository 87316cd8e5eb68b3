#!/bin/bash
# Round 5: the one-launch WAL scan's phase-A threshold (first records of
# units >= AMIN walked before the framing ends): 2,049 (product) vs 4,096 /
# 8,192 / 16,384, --wal-path 1, two interleaved reps.  usage: tools/r05_amin.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05amin}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
for a in 4096 8192 16384; do bash tools/build_variant.sh a$a -DLVK_PIPE_AMIN=$a >> "$out/build.txt" 2>&1 || exit 1; done
bash tools/build_variant.sh sf -DLVK_PIPE_B_SMALL_FIRST=1 >> "$out/build.txt" 2>&1 || exit 1
bash tools/build_variant.sh sf16k -DLVK_PIPE_B_SMALL_FIRST=1 -DLVK_PIPE_AMIN=16384 >> "$out/build.txt" 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --wal-device --wal-path 1 --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" || exit 1
  for a in a4096 a8192 a16384 sf sf16k; do
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_$a.so timeout -k 10 200 python3 bench.py --wal-device --wal-path 1 \
      --cpu-seconds 0 > "$out/${a}_$r.json" 2>> "$out/err.txt" || exit 1
  done
done
for f in "$out"/*_*.json; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['roofline']['frac'], d['roofline']['ms_avg'])" "$f"; done
echo "all steps done"
