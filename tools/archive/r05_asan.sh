#!/bin/bash
# Round 5: the host code of every unit -- the .cc files and the host side of
# the .hip files (the pipelined WAL scan's worker) -- under AddressSanitizer
# on the GPU box: the WAL tests and a repeated pipelined-scan stress.
# usage: tools/r05_asan.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05asan}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
make -s -C leveldb-rs_amd sanitize_hip > "$out/build.txt" 2>&1 || exit 1
export out
export LVGPU_EXPERIMENT=1 LVGPU_LIB=$root/leveldb-rs_amd/lib/variants/liblvgpu_asanhip.so
export ASAN_OPTIONS=detect_leaks=0:log_path=$out/asan_report
AS="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libstdc++.so)"  # (libstdc++ first: ASan intercepts __cxa_throw)
LD_PRELOAD=$AS timeout -k 10 400 python3 -X faulthandler -u -m pytest tests/test_gpu_wal.py tests/test_wal_log.py -m gpu -k "not device" -x -q \
  --timeout 300 --timeout-method thread > "$out/pytest.txt" 2>&1 &&
LD_PRELOAD=$AS timeout -k 10 400 python3 -X faulthandler -u tools/pipe_stress.py 12 > "$out/stress.txt" 2>&1 &&
echo "asan steps done"
