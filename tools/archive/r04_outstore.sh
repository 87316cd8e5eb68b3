#!/bin/bash
# Round 4 timing probe: the class kernel's output stores -- product (each CRC
# to its buffer's slot: scattered dwords), sortedout (to its sorted position:
# 16-B runs; LVK_EXP_SORTEDOUT, wrong order, timing only) and noout (none) --
# on the whole C2 / C4 batches.  usage: tools/r04_outstore.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/outstore}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
bash tools/build_variant.sh sortedout -DLVK_EXP_SORTEDOUT=1 > "$out/build.txt" 2>&1 &&
bash tools/build_variant.sh noout -DLVK_EXP_NOOUT=1 >> "$out/build.txt" 2>&1 || exit 1
F="--cpu-seconds 0 --traffic off --c5-strong off"
for r in 1 2; do
  for w in c2 c4; do
    timeout -k 10 200 python3 bench.py --workload $w --api offsets $F > "$out/${w}_prod_$r.json" 2>> "$out/err.txt" &&
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_sortedout.so timeout -k 10 200 python3 bench.py --workload $w --api offsets $F \
      > "$out/${w}_sortedout_$r.json" 2>> "$out/err.txt"
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_noout.so timeout -k 10 200 python3 bench.py --workload $w --api offsets $F \
      > "$out/${w}_noout_$r.json" 2>> "$out/err.txt"
  done
done
echo "all steps done"
