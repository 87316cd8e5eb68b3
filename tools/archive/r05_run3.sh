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
# (stdout: the key lines, in case gpurun_out is not copied back)
for f in "$out"/wal/wal_device.json "$out"/hash/prod_1.json "$out"/hash/g2_1.json; do tail -c 600 "$f"; echo; done
python3 -c "import json; d=json.load(open('$out/wal/trace/trace.json')); print({k: d[k] for k in ('end','own_done_last_wave','walk_done_first_wave','walk_done_last_wave')})" || true
