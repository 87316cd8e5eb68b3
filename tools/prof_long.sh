#!/bin/bash
# Kernel split of the few-long-buffer offsets calls (tools/long_offsets_probe.py
# under rocprofv3 --kernel-trace --stats): per kernel, the steady mean of the
# last 50 launches.  usage: tools/prof_long.sh OUTDIR [N:BYTES ...]
# (LONG_API=lib: the library workspace instead of a caller workspace)
set -o pipefail
out=${1:-gpurun_out/prof_long}; shift
cases=${*:-1:16777216 1024:65536 16:1048576}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
for c in $cases; do
  n=${c%%:*}; b=${c#*:}
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/$out/k_${n}x$b" -o p -- \
      python3 "$root/tools/long_offsets_probe.py" "$n" "$b" "${LONG_API:-ws}") > "$out/k_${n}x$b.log" 2>&1 || { echo "case $c failed"; tail -5 "$out/k_${n}x$b.log"; exit 1; }
  grep "us per call" "$out/k_${n}x$b.log"
  python3 tools/kstats_steady.py "$(ls "$out/k_${n}x$b"/*kernel_trace.csv | head -n 1)" 50 "$out/${n}x${b}_steady.json" | \
    python3 -c "import json,sys; d=json.load(sys.stdin); print('  ', ', '.join(f'{k.split(\"::\")[-1][:40]} {v[\"mean_us\"]}' for k, v in d.items()))"
  rm -rf "$out/k_${n}x$b"
done
