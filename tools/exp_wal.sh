#!/bin/bash
# WAL device-scan timing variants (experiment builds, -D flags; wrong CRCs allowed): builds them on the box, runs
# bench.py --wal-device under each.   tools/exp_wal.sh OUT "name:flags ..."
set -o pipefail
out=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$out"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  if [ "$name" != base ]; then
    timeout -k 10 200 "$root/tools/build_variant.sh" "$name" $flags > "$out/build_$name.log" 2>&1 || exit 1
    env="LVGPU_EXPERIMENT=1 LVGPU_LIB=$root/leveldb-rs_amd/lib/variants/liblvgpu_$name.so"
  else
    env=""
  fi
  env $env timeout -k 10 200 python3 "$root/bench.py" --wal-device > "$out/$name.json" 2> "$out/$name.err" || exit 1
  python3 -c "import json; d=json.load(open('$out/$name.json')); r=d['roofline']; print('$name', r['ms_avg'], r['frac'])"
done
