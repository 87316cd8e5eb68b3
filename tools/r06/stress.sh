#!/bin/bash
# Round 6 final tree: the randomised parity sweeps at scale (SST seal / verify
# walk changed this round: runs of four blocks per group).
set -o pipefail
out=${1:-gpurun_out/r06stress}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
t() { timeout -k 10 "$1" python3 -u -m pytest "$2" -q -m gpu --timeout 120 --timeout-method thread > "$out/$3" 2>&1; }
LVGPU_SST_STRESS_TRIALS=3000 t 300 tests/test_gpu_table_stress.py sst_3000.txt &&
LVGPU_WAL_STRESS_TRIALS=3000 t 300 tests/test_gpu_wal_stress.py wal_3000.txt &&
LVGPU_HASH_STRESS_TRIALS=2000 t 200 tests/test_gpu_hash_stress.py hash_2000.txt &&
LVGPU_STRESS_TRIALS=5000 t 400 tests/test_gpu_stress.py offsets_5000.txt &&
for f in "$out"/*.txt; do echo "$f: $(tail -n 1 "$f")"; done
