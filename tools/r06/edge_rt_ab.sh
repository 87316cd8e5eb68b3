#!/bin/bash
# Round 6 (final): the aligned-row walk (G = 16: the class kernel's long
# buffers, the WAL scan, the table walk) loading each round's first and last
# batch with the default (L2-allocating) policy instead of non-temporal
# (LVK_EDGE_RT=1), so a 128-B line shared by two neighbouring buffers is
# fetched once, against the product.
# (Results in profiles/r06/edge_rt/; the knob lived in 3f58364 and was reverted.)
set -o pipefail
out=${1:-gpurun_out/r06edge}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
bash tools/build_variant.sh edge -DLVK_EDGE_RT=1 > "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_edge.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/pytest_edge.txt" 2>&1 || exit 1
B="--cpu-seconds 0 --traffic off --c5-strong off"
for r in 1 2; do
  for v in prod edge; do
    if [ $v = edge ]; then export LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_edge.so; else unset LVGPU_EXPERIMENT LVGPU_LIB; fi
    timeout -k 10 200 python3 bench.py --workload c2 --api offsets $B > "$out/${v}_c2_$r.json" 2>> "$out/err.txt" || exit 1
    timeout -k 10 200 python3 bench.py --workload c4 --api offsets $B > "$out/${v}_c4_$r.json" 2>> "$out/err.txt" || exit 1
    timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/${v}_table_$r.json" 2>> "$out/err.txt" || exit 1
    timeout -k 10 200 python3 bench.py --wal-device --cpu-seconds 0 --traffic off > "$out/${v}_wal_$r.json" 2>> "$out/err.txt" || exit 1
  done
done
unset LVGPU_EXPERIMENT LVGPU_LIB
for f in "$out"/*_c2_*.json "$out"/*_c4_*.json "$out"/*_wal_*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['roofline']['frac'], d.get('ms_per_step'))" "$f"; done
for f in "$out"/*_table_*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['seal']['frac_of_8TBps'], d['verify']['frac_of_8TBps'])" "$f"; done
