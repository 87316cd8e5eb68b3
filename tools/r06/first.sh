#!/bin/bash
# Round 6, first GPU pass: the WAL device tests after the one-launch path's
# removal, the --wal-device line with per-kernel FETCH/WRITE, and the
# exit-time probe under rocprofv3.
set -o pipefail
out=${1:-gpurun_out/r06first}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wal.py tests/test_gpu_wal_stress.py -x -q --timeout 120 --timeout-method thread > "$out/pytest_wal.txt" 2>&1 &&
timeout -k 10 300 python3 bench.py --wal-device --cpu-seconds 0 > "$out/wal_device.json" 2> "$out/wal_device.err" &&
(cd /tmp && timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --output-format csv -d "$root/$out/pmc_wal" -o pmc -- python3 "$root/bench.py" --wal-device --cpu-seconds 0 --steps 20 --warmup 10 --no-settle) > "$out/pmc_wal.log" 2>&1 &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/$out/prof_wal" -o wal -- python3 "$root/bench.py" --wal-device --steps 50 --warmup 20 --cpu-seconds 0) > "$out/prof_wal.log" 2>&1 &&
python3 tools/kstats_steady.py "$(ls "$out/prof_wal"/*kernel_trace.csv | head -n 1)" 50 "$out/prof_wal_steady.json" > /dev/null &&
for w in device host pipe; do
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/$out/exit_$w" -o e -- python3 "$root/tools/r06/exit_probe.py" $w) > "$out/exit_$w.log" 2>&1
  rc=$?
  echo "exit_probe $w rc=$rc" >> "$out/exit_rc.txt"
  [ $rc -eq 0 ] || break  # a crash ends the GPU work of this call
done
find "$out" -name '*kernel_trace.csv' -size +1M -delete
echo done
