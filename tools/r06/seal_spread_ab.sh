#!/bin/bash
# Round 6 (final): the seal's trailer stores spread over the walk instead of
# one flush per wave at its end (LVK_SEAL_FLUSH=4: every 4 rounds), with the
# load-free flush (LVK_SEAL_NARROW=1), and with or without non-temporal
# stores (LVK_SEAL_NT=1), against the product.  The no-store timing study
# (seal_nostore_probe.sh) put the trailer stores at ~10 us of ~200.
# (Results in profiles/r06/seal_spread/; the knobs lived in 02e8055 and were reverted.)
set -o pipefail
out=${1:-gpurun_out/r06sp}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
bash tools/build_variant.sh nn4 -DLVK_SEAL_NARROW=1 -DLVK_SEAL_NT=1 -DLVK_SEAL_FLUSH=4 > "$out/build.txt" 2>&1 || exit 1
bash tools/build_variant.sh nn16 -DLVK_SEAL_NARROW=1 -DLVK_SEAL_NT=1 >> "$out/build.txt" 2>&1 || exit 1
bash tools/build_variant.sh n4 -DLVK_SEAL_NARROW=1 -DLVK_SEAL_FLUSH=4 >> "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
for v in nn4 n4; do
  LVGPU_SST_STRESS_TRIALS=200 LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_table.py tests/test_gpu_table_stress.py -x -q --timeout 120 --timeout-method thread > "$out/pytest_$v.txt" 2>&1 || exit 1
done
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" || exit 1
  for v in nn4 nn16 n4; do
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_$v.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/${v}_$r.json" 2>> "$out/err.txt" || exit 1
  done
done
for f in "$out"/prod_*.json "$out"/nn4_*.json "$out"/nn16_*.json "$out"/n4_*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['seal']['frac_of_8TBps'], d['seal']['ms_avg'], d['verify']['frac_of_8TBps'])" "$f"; done
