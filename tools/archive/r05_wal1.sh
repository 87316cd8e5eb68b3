#!/bin/bash
# Round 5: the one-launch WAL scan (wal_pipe_kernel).  The WAL GPU tests (both
# device paths), the reference LogTest suite on the GPU backend, the
# --wal-device line, and its rocprof kernel stats.  usage: tools/r05_wal1.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05w}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wal.py tests/test_wal_log.py -m gpu -x -v --timeout 120 \
  --timeout-method thread > "$out/pytest.txt" 2>&1 &&
timeout -k 10 300 python3 bench.py --wal-device --cpu-seconds 0 > "$out/wal_device.json" 2> "$out/wal_device.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o wal -- python3 bench.py --wal-device --cpu-seconds 0 \
  > "$out/prof_wal.json" 2> "$out/prof_wal.err" &&
echo "all steps done"
