#!/bin/bash
# Round 5, second check: the WAL one-launch scan first (its tests, its bench
# line and rocprof stats), then the whole GPU suite, smoke, sweep / long, the
# pack probe and the world-size-8 gloo rehearsal.  usage: tools/r05_check2.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05b}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
bash tools/r05_wal1.sh "$out/wal" &&
bash tools/r05_check1.sh "$out/check"
