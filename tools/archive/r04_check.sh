#!/bin/bash
# Round-4 GPU check: the GPU suite (incl. the full-size strong C5 test), smoke,
# the driver-flag bench line (with its c5_strong sub-record) and the N=2 gloo
# rehearsal of the same line.  Each GPU step has its own limit; the chain
# stops at the first failure.
# usage: tools/r04_check.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r04}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/pytest.txt" 2>&1 &&
echo "pytest done" &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 &&
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > "$out/default_driver.json" 2> "$out/default_driver.err" &&
echo "bench done" &&
LVGPU_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 20 --warmup 5 --cpu-seconds 2 > "$out/gloo2.json" 2> "$out/gloo2.err" &&
echo "gloo done" &&
timeout -k 10 300 python3 bench.py --hash > "$out/hash.json" 2> "$out/hash.err" &&
timeout -k 10 300 python3 bench.py --table > "$out/table.json" 2> "$out/table.err" &&
timeout -k 10 300 python3 bench.py --wal-device > "$out/wal_device.json" 2> "$out/wal_device.err" &&
timeout -k 10 300 python3 bench.py --wal > "$out/wal.json" 2> "$out/wal.err" &&
timeout -k 10 300 python3 bench.py --long > "$out/long.json" 2> "$out/long.err" &&
echo "all steps done"
