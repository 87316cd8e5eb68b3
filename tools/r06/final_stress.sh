#!/bin/bash
# Round 6, last tree: the GPU suite, smoke(), and the randomised parity
# sweeps at 4x the earlier pass (trial i uses seed base + i, so these
# include the earlier 13,000 and add new ones).
set -o pipefail
out=${1:-gpurun_out/r06fs}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
t() { timeout -k 10 "$1" python3 -u -m pytest "$2" -q -m gpu --timeout 120 --timeout-method thread > "$out/$3" 2>&1; }
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_suite.txt" 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.txt" 2>&1 &&
LVGPU_HASH_STRESS_TRIALS=8000 t 120 tests/test_gpu_hash_stress.py hash_8000.txt &&
LVGPU_WAL_STRESS_TRIALS=12000 t 240 tests/test_gpu_wal_stress.py wal_12000.txt &&
LVGPU_SST_STRESS_TRIALS=12000 t 360 tests/test_gpu_table_stress.py sst_12000.txt &&
LVGPU_STRESS_TRIALS=12000 t 480 tests/test_gpu_stress.py offsets_12000.txt &&
for f in "$out"/*.txt; do echo "$f: $(tail -n 1 "$f")"; done
