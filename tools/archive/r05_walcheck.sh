#!/bin/bash
# The WAL one-launch scan: its tests (both device paths, the pipelined host
# scan), the --wal-device and --wal lines, the phase timeline variant.  usage: tools/r05_walcheck.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05w}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wal.py tests/test_wal_log.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > "$out/pytest.txt" 2>&1 &&
timeout -k 10 300 python3 bench.py --wal-device --cpu-seconds 0 > "$out/wal_device.json" 2> "$out/wal_device.err" &&
timeout -k 10 600 python3 bench.py --wal --cpu-seconds 0 > "$out/wal_host.json" 2> "$out/wal_host.err" &&
bash tools/r05_waltrace.sh "$out/trace" &&
echo "all steps done"
