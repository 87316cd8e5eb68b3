#!/bin/bash
# Round 6, second GPU pass: launch-overhead probe; --wal-device kernel stats
# and FETCH / WRITE per kernel (separate passes); the LVK_WAL_UNSORT=0 variant
# (class kernel stores log-order CRCs directly) A/B; the exit probe under
# rocprofv3; bench --wal x3 (recovery spread, pageable and pinned logs).
set -o pipefail
out=${1:-gpurun_out/r06p2}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
timeout -k 10 60 ./tools/launch_probe > "$out/launch_probe.json" 2>&1 || exit 1
bash tools/prof_8f.sh "$out/prof" wal > "$out/prof.log" 2>&1 || exit 1
bash tools/build_variant.sh nounsort -DLVK_WAL_UNSORT=0 > "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --wal-device --cpu-seconds 0 > "$out/wal_prod_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_nounsort.so timeout -k 10 200 python3 bench.py --wal-device --cpu-seconds 0 > "$out/wal_nounsort_$r.json" 2>> "$out/err.txt" || exit 1
done
for w in device host pipe; do
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/$out/exit_$w" -o e -- python3 "$root/tools/r06/exit_probe.py" $w) > "$out/exit_$w.log" 2>&1
  rc=$?
  echo "exit_probe $w rc=$rc" >> "$out/exit_rc.txt"
  [ $rc -eq 0 ] || exit 1  # a crash ends the GPU work of this call
done
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 > "$out/wal_$r.json" 2> "$out/wal_$r.err" || exit 1
done
find "$out" -name '*kernel_trace.csv' -size +1M -delete
echo pass2 done
