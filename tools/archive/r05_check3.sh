#!/bin/bash
# usage: tools/r05_check3.sh OUTDIR -- the wal_pipe timeline, then the check-1 set
set -o pipefail
out=${1:-gpurun_out/r05c}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
bash tools/r05_waltrace.sh "$out/trace" && bash tools/r05_check1.sh "$out/check"
