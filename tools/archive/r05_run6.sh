#!/bin/bash
# Round 5: the restored WAL one-launch scan (tests, --wal-device), the host
# pipelined scan under glibc heap checks and under ASan (host code of every
# unit), then the full check (GPU suite, smoke, sweep, long, pack probe,
# gloo8).  usage: tools/r05_run6.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05r7}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 -X faulthandler -u -m pytest tests/test_gpu_wal.py tests/test_wal_log.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > "$out/pytest_wal.txt" 2>&1 &&
timeout -k 10 300 python3 bench.py --wal-device --cpu-seconds 0 > "$out/wal_device.json" 2> "$out/wal_device.err" &&
tail -c 300 "$out/wal_device.json" && echo &&
MALLOC_CHECK_=3 timeout -k 10 400 python3 -X faulthandler -u tools/pipe_stress.py 16 > "$out/stress_malloccheck.txt" 2>&1
echo "stress (malloc check) rc=$?"; tail -3 "$out/stress_malloccheck.txt"
bash tools/r05_asan.sh "$out/asan"
echo "asan rc=$?"; tail -3 "$out/asan/pytest.txt"; tail -3 "$out/asan/stress.txt" 2>/dev/null; ls "$out/asan"
bash tools/r05_check1.sh "$out/check" && tail -3 "$out/check/pytest.txt" && cat "$out/check/smoke.txt" &&
echo "all steps done"
