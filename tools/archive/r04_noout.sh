#!/bin/bash
# Round 4 timing probe: what the class kernel's scattered output stores cost
# (variant noout: LVK_EXP_NOOUT=1, CRCs computed but not stored -- timing
# only, no parity) on C2 / C4 / C3 via offsets / the WAL scan.
# usage: tools/r04_noout.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/noout}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
bash tools/build_variant.sh noout -DLVK_EXP_NOOUT=1 > "$out/build.txt" 2>&1 || exit 1
F="--cpu-seconds 0 --traffic off --c5-strong off"
for r in 1 2; do
  for w in c2 c4; do
    timeout -k 10 200 python3 tools/class_split_probe.py $w 40 > "$out/${w}_prod_$r.txt" 2>> "$out/err.txt" &&
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_noout.so timeout -k 10 200 python3 tools/class_split_probe.py $w 40 \
      > "$out/${w}_noout_$r.txt" 2>> "$out/err.txt" || exit 1
  done
done &&
echo "all steps done"
