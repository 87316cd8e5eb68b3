#!/bin/bash
# Round 6 (2nd): the seal with a trailer-writer wave (LVK_SEAL_WRITER=1: 15
# walkers publish their staged trailers, wave 15 writes them) against the
# product, interleaved, plus the table tests on the variant.
# (The knob lived in commit a2dd333 only; check that commit out to rerun.)
set -o pipefail
out=${1:-gpurun_out/r06sw}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
bash tools/build_variant.sh writer -DLVK_SEAL_WRITER=1 > "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_writer.so timeout -k 10 300 python3 -u -m pytest tests/test_table.py tests/test_gpu_table_stress.py -x -q --timeout 120 --timeout-method thread > "$out/pytest_writer.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/prod_$r.json" 2>> "$out/err.txt" || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_writer.so timeout -k 10 200 python3 bench.py --table --cpu-seconds 0 > "$out/writer_$r.json" 2>> "$out/err.txt" || exit 1
done
for f in "$out"/prod_*.json "$out"/writer_*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['seal']['frac_of_8TBps'], d['verify']['frac_of_8TBps'])" "$f"; done
