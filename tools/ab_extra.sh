#!/bin/bash
# A/B of library variants on the table-trailer bench (bench.py --table):
#   tools/ab_extra.sh OUT "variantA variantB ..."
set -o pipefail
out=$1; vars=$2; shift 2
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$out"
for v in $vars; do
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$root/leveldb-rs_amd/lib/variants/liblvgpu_$v.so timeout -k 10 300 python3 bench.py --table "$@" \
    > "$out/${v}_table.json" 2> "$out/${v}_table.err" || exit 1
  python3 -c "import json; d=json.load(open('$out/${v}_table.json')); print('$v table seal', d['seal']['frac_of_8TBps'], 'verify', d['verify']['frac_of_8TBps'])"
done
