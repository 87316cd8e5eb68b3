#!/bin/bash
# bench.py --long under the product library and experiment variants (built on
# the box):  tools/ab_long.sh OUT "name:flags ..." (name "base" = product).
set -o pipefail
out=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$out"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  env=""
  if [ "$name" != base ]; then
    timeout -k 10 200 "$root/tools/build_variant.sh" "$name" $flags > "$out/build_$name.log" 2>&1 || exit 1
    env="LVGPU_EXPERIMENT=1 LVGPU_LIB=$root/leveldb-rs_amd/lib/variants/liblvgpu_$name.so"
  fi
  env $env timeout -k 10 200 python3 "$root/bench.py" --long > "$out/$name.json" 2> "$out/$name.err" || exit 1
  python3 -c "
import json
l=[x for x in open('$out/$name.json') if x.startswith('{') and 'results' in x][-1]
d=json.loads(l)
print('$name', ' '.join(f\"{r['blocks']}x{r['block_bytes']>>10}K s={r['strided']['us_avg']} o={r['offsets']['us_avg']}\" for r in d['results']))"
done
