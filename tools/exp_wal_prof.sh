#!/bin/bash
# WAL device-scan kernel split under library variants (experiment builds,
# wrong CRCs allowed): builds each on the box, runs bench.py --wal-device under
# rocprofv3 --kernel-trace and prints the steady per-kernel means.
#   tools/exp_wal_prof.sh OUT "name:-DFOO=1,-DBAR=2" ...     (name "base": the product library)
set -o pipefail
out=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$root/$out"
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  envs=()
  if [ "$name" != base ]; then
    timeout -k 10 200 bash "$root/tools/build_variant.sh" "$name" ${flags//,/ } > "$root/$out/build_$name.log" 2>&1 || exit 1
    envs=(LVGPU_EXPERIMENT=1 "LVGPU_LIB=$root/leveldb-rs_amd/lib/variants/liblvgpu_$name.so")
  fi
  (cd /tmp && env "${envs[@]}" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$root/$out/$name" -o p -- python3 "$root/bench.py" --wal-device --steps 50 --warmup 20) \
     > "$root/$out/$name.txt" 2>&1 || exit 1
  echo "== $name $(grep -o '"frac": [0-9.]*, "ms_avg": [0-9.]*' "$root/$out/$name.txt" | head -n 1)"
  python3 "$root/tools/kstats_steady.py" "$(ls "$root/$out/$name"/*kernel_trace.csv | head -n 1)" 50 \
    "$root/$out/${name}_steady.json" | python3 -c "import json,sys; d=json.load(sys.stdin); print('\n'.join(f'  {k[:60]:60s} {v[\"mean_us\"]}' for k,v in d.items()))"
  find "$root/$out/$name" -name '*kernel_trace.csv' -size +1M -delete
done
