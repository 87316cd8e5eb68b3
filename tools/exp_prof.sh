#!/bin/bash
# Kernel-trace stats of bench workloads under library variants.
#   tools/exp_prof.sh OUT "variantA variantB" "c2 c4 c3" [extra bench args]
set -o pipefail
out=$1; vars=$2; works=$3; shift 3
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$root/$out"
export TMPDIR=/tmp
for v in $vars; do
  for w in $works; do
    (cd /tmp && LVGPU_EXPERIMENT=1 LVGPU_LIB=$root/leveldb-rs_amd/lib/variants/liblvgpu_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
       --output-format csv -d "$root/$out/${v}_$w" -o p -- python3 "$root/bench.py" --workload $w --api offsets \
       --steps 50 --warmup 50 --cpu-seconds 0 --traffic off "$@") > "$root/$out/${v}_$w.txt" 2>&1 || exit 1
    echo "== $v $w"; cut -d, -f1-4 "$root/$out/${v}_$w"/p_kernel_stats.csv | cut -c1-150 | grep -v "fill\|elementwise\|Fill" 
  done
done
