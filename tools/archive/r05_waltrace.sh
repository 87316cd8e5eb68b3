#!/bin/bash
# wal_pipe_kernel phase timeline (timing variant), usage: tools/r05_waltrace.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05t}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
bash tools/build_variant.sh walptrace -DLVK_WAL_PIPE_TRACE=1 > "$out/build.txt" 2>&1 &&
LVGPU_EXPERIMENT=1 LVGPU_LIB=$root/leveldb-rs_amd/lib/variants/liblvgpu_walptrace.so \
  timeout -k 10 300 python3 tools/wal_pipe_trace.py 5 > "$out/trace.json" 2> "$out/trace.err" &&
echo "all steps done"
