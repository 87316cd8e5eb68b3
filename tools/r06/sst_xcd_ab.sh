#!/bin/bash
# Round 6 (2nd): SST table walk with adjacent claims on one XCD
# (LVK_SST_XCD=1) against the product, interleaved, plus the table tests on
# the variant and a FETCH_SIZE pass of each.
# (The knob lived in commit 3da572a only; check that commit out to rerun.)
set -o pipefail
out=${1:-gpurun_out/r06xcd}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
bash tools/build_variant.sh xcd -DLVK_SST_XCD=1 > "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_xcd.so timeout -k 10 300 python3 -u -m pytest tests/test_table.py tests/test_gpu_table_stress.py -x -q --timeout 120 --timeout-method thread > "$out/pytest_xcd.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_xcd.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/xcd_$r.json" 2>> "$out/err.txt" || exit 1
done
for v in prod xcd; do
  if [ $v = xcd ]; then export LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_xcd.so; fi
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$root/$out/pmc_$v" -o pmc -- \
     python3 "$root/bench.py" --table --steps 10 --warmup 5 --cpu-seconds 0 --no-settle) > "$out/pmc_$v.log" 2>&1 || exit 1
done
unset LVGPU_EXPERIMENT LVGPU_LIB
for f in "$out"/prod_*.json "$out"/xcd_*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['seal']['frac_of_8TBps'], d['verify']['frac_of_8TBps'])" "$f"; done
for v in prod xcd; do python3 -c "
import sys; sys.path.insert(0, '.')
import importlib.util, glob
spec = importlib.util.spec_from_file_location('b', 'bench.py'); b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)
f = glob.glob('$out/pmc_$v/**/*counter_collection.csv', recursive=True)[0]
print('$v', {k: round(x / 1e6, 1) for k, x in b.read_pmc_per_kernel(f, 'FETCH_SIZE').items()})"; done
