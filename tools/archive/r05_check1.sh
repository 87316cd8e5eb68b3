#!/bin/bash
# Round 5, first check: GPU suite (hint checks, ADVICE join fix, pack cache),
# smoke, the sweep and long-buffer lines (the aligned-hint path with its
# length/offset checks against the strided API on the same box), and the
# multi-device pack probe, and the world-size-8 rehearsal (8 gloo ranks on
# the box's one GPU, the driver's N = 8 line).  usage: tools/r05_check1.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05a}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/pytest.txt" 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.txt" 2>&1 &&
timeout -k 10 400 python3 bench.py --sweep > "$out/sweep.json" 2> "$out/sweep.err" &&
timeout -k 10 300 python3 bench.py --long > "$out/long.json" 2> "$out/long.err" &&
timeout -k 10 200 python3 tools/multi_pack_probe.py 10 > "$out/multi_pack.json" 2> "$out/multi_pack.err" &&
mkdir -p "$out/gloo8" &&
LVGPU_BENCH_BACKEND=gloo timeout -k 10 900 python3 bench.py --gpus 8 --steps 20 --warmup 5 > "$out/gloo8/bench.json" 2> "$out/gloo8/bench.err" &&
echo "all steps done"
