#!/bin/bash
# A/B experiment: bench workloads under several library variants.
#   tools/exp_ab.sh OUT "variantA variantB" "c2 c4 c3" [extra bench args]
set -o pipefail
out=$1; vars=$2; works=$3; shift 3
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$out"
for v in $vars; do
  for w in $works; do
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$root/leveldb-rs_amd/lib/variants/liblvgpu_$v.so timeout -k 10 300 \
      python3 bench.py --workload $w --api ${API:-offsets} --cpu-seconds 0 "$@" > "$out/${v}_$w.json" 2> "$out/${v}_$w.err" || exit 1
    python3 -c "import json,sys; d=json.load(open('$out/${v}_$w.json')); r=d['roofline']; print('$v $w', d['value'], r['achieved'], r['frac'], r.get('traffic'), d['config']['bytes_per_gpu'])"
  done
done
