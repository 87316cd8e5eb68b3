#!/bin/bash
# Round 4, last check on the final tree: GPU suite, smoke, 200-trial sweep,
# the driver-flag default line, and the C2 / C4 / WAL lines with their CPU
# baselines and parity samples.  usage: tools/r04_check4.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r04d}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/pytest.txt" 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.txt" 2>&1 &&
LVGPU_STRESS_TRIALS=200 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_stress.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > "$out/stress200.txt" 2>&1 &&
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > "$out/default_driver.json" 2> "$out/default_driver.err" &&
timeout -k 10 400 python3 bench.py --workload c2 --api offsets --cpu-seconds 5 > "$out/c2.json" 2> "$out/c2.err" &&
timeout -k 10 400 python3 bench.py --workload c4 --api offsets --cpu-seconds 5 > "$out/c4.json" 2> "$out/c4.err" &&
timeout -k 10 300 python3 bench.py --wal-device > "$out/wal_device.json" 2> "$out/wal_device.err" &&
echo "all steps done"
