#!/bin/bash
# Round 6 (final), timing study: the seal with its trailer stores skipped
# (LVK_SEAL_NOSTORE=1, wrong output by design; bench.py skips parity for
# experiment variants) against the product -- what any change to how the
# trailers are written could gain at most.
# (Results in profiles/r06/seal_nostore/; the knobs lived in 02e8055 and were reverted.)
set -o pipefail
out=${1:-gpurun_out/r06ns}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
bash tools/build_variant.sh ns -DLVK_SEAL_NOSTORE=1 > "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_ns.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/ns_$r.json" 2>> "$out/err.txt" || exit 1
done
for f in "$out"/prod_*.json "$out"/ns_*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['seal']['frac_of_8TBps'], d['seal']['ms_avg'], d['verify']['frac_of_8TBps'])" "$f"; done
