#!/bin/bash
# Round 6 (2nd): does the per-launch gap depend on where the HIP runtime puts
# kernel arguments?  launch_probe and the default C3 line under
# HIP_FORCE_DEV_KERNARG=0 / 1, interleaved.
set -o pipefail
out=${1:-gpurun_out/r06ka}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
for v in 0 1; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 tools/launch_probe > "$out/probe_ka$v.json" || exit 1
done
for r in 1 2; do
  for v in 0 1; do
    HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python3 bench.py --steps 200 --warmup 100 --cpu-seconds 0 --traffic off --c5-strong off > "$out/c3_ka${v}_$r.json" 2>> "$out/err.txt" || exit 1
  done
done
for f in "$out"/c3_*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['frac'])" "$f"; done
cat "$out"/probe_ka*.json
