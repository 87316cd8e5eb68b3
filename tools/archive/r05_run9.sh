#!/bin/bash
# Round 5: the world-size-8 rehearsal (8 gloo ranks on the box's one GPU,
# the driver's N = 8 line: C3 and c5_strong with every rank's parity sample),
# a 1-GPU default line, then the one-launch WAL scan's phase-A threshold sweep.
# usage: tools/r05_run9.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05r10}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out/gloo8"
export TMPDIR=/tmp
LVGPU_BENCH_BACKEND=gloo timeout -k 10 900 python3 bench.py --gpus 8 --steps 20 --warmup 5 > "$out/gloo8/bench.json" 2> "$out/gloo8/bench.err" &&
python3 -c "
import json
d=json.loads(open('$out/gloo8/bench.json').read().strip().splitlines()[-1])
c=d['c5_strong']
print('world', d['world_size'], 'C3 per_gpu', len(d['per_gpu']), [p.get('parity_sample') for p in d['per_gpu']])
print('c5 per_gpu', len(c['per_gpu']), [p.get('parity_sample') for p in c['per_gpu']], c['value'])" &&
bash tools/r05_amin.sh "$out/amin" | tail -10 &&
echo "all steps done"
