#!/bin/bash
# Kernel evidence for the SURVEY 8f rows: rocprofv3 kernel-trace stats (and
# the steady mean of the last 50 launches) plus separate PMC passes for
# FETCH_SIZE and WRITE_SIZE (one counter per pass, kernel counters only) of
# the SST seal/verify kernels (bench.py --table), the hash kernel (--hash)
# and the device WAL scan (--wal-device).  Each GPU step has its own time
# limit; the chain stops at the first failure.
# usage: tools/prof_8f.sh OUTDIR [table hash wal]
set -o pipefail
out=${1:-gpurun_out/prof8f}; shift
what=${*:-table hash wal}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
declare -A ARGS=([table]="--table" [hash]="--hash" [wal]="--wal-device")
k() { local name=$1; shift
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/$out/k_$name" -o "$name" -- \
          python3 "$root/bench.py" "$@" --steps 50 --warmup 20 --cpu-seconds 0) > "$out/k_$name.log" 2>&1 &&
      python3 tools/kstats_steady.py "$(ls "$out/k_$name"/*kernel_trace.csv | head -n 1)" 50 "$out/${name}_steady.json" > /dev/null &&
      cp "$(ls "$out/k_$name"/*kernel_stats.csv | head -n 1)" "$out/${name}_kernel_stats.csv"; }
m() { local name=$1 ctr=$2; shift 2
      (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc "$ctr" --output-format csv -d "$root/$out/m_$name/$ctr" -o pmc -- \
          python3 "$root/bench.py" "$@" --steps 5 --warmup 1 --no-settle --cpu-seconds 0) > "$out/m_${name}_$ctr.log" 2>&1; }
for w in $what; do
  a=${ARGS[$w]}
  k "$w" $a && m "$w" FETCH_SIZE $a && m "$w" WRITE_SIZE $a &&
  python3 tools/pmc_summary.py "$out/m_$w" "$out/${w}_pmc.json" > /dev/null || { echo "step $w failed"; exit 1; }
  rm -rf "$out/k_$w" "$out/m_$w"
  echo "$w done"
done
