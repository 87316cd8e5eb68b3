#!/bin/bash
# Round 4: the session-start hash kernel with only its metadata prefetch made
# exact (every lane loads, clamped; validity applied when the set is used),
# against the session-start build (abtmp/, variant "base") and the product
# switch off (variant "pf0").  Hash tests, then the hash bench alternated.
# usage: tools/r04_hash_exact.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/hash_exact}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
timeout -k 10 300 python3 -u -m pytest tests/test_hash.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$out/pytest_hash.txt" 2>&1 &&
(cd abtmp/leveldb-rs_amd && make -j16 lib/liblvgpu.so > "$root/$out/build.txt" 2>&1) && mkdir -p "$VD" &&
cp abtmp/leveldb-rs_amd/lib/liblvgpu.so "$VD/liblvgpu_base.so" &&
bash tools/build_variant.sh pf0 -DLVK_HASH_PREFETCH_EXACT=0 >> "$out/build.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_base.so timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 \
    > "$out/base_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_pf0.so timeout -k 10 200 python3 bench.py --hash --cpu-seconds 0 \
    > "$out/pf0_$r.json" 2>> "$out/err.txt" || exit 1
done &&
echo "all steps done"
