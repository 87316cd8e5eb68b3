#!/bin/bash
# Round 5: SST seal variants (4 rows per batch on the G = 16 image; 8 rounds
# per trailer flush) against the product, two interleaved reps; then the hash
# line (its VALU pass classifies kernels by template argument now).
# usage: tools/r05_sst.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05sst}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
bash tools/build_variant.sh s4 -DLVK_SEAL_ROWS=4 > "$out/build.txt" 2>&1 || exit 1
bash tools/build_variant.sh sf8 -DLVK_SEAL_FLUSH=8 >> "$out/build.txt" 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" || exit 1
  for v in s4 sf8; do
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_$v.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 \
      > "$out/${v}_$r.json" 2>> "$out/err.txt" || exit 1
  done
done
for f in "$out"/*_[12].json; do python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], 'seal', d['seal']['frac_of_8TBps'], 'verify', d['verify']['frac_of_8TBps'])" "$f"; done
timeout -k 10 400 python3 bench.py --hash > "$out/hash.json" 2> "$out/hash.err" || exit 1
python3 -c "
import json; d=json.loads(open('$out/hash.json').read().strip().splitlines()[-1])
print('hash', d['roofline'].get('bound'), d['roofline'].get('frac'), 'valu', d.get('roofline_valu'))"
echo "all steps done"
