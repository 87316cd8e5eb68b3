#!/bin/bash
# Round 5: the WAL one-launch scan with cross-workgroup phase-B rounds (tests,
# --wal-device, --wal, timeline), then the hash LDS-DMA A/B and the VALU
# counter calibration.  usage: tools/r05_run3.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05r3}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
bash tools/r05_walcheck.sh "$out/wal" &&
bash tools/r05_hash2.sh "$out/hash" &&
bash tools/r05_valu.sh "$out/valu" &&
echo "all steps done"
