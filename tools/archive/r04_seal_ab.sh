#!/bin/bash
# (Run once in round 4, profiles/r04/ab1/; the switch it measured was then retired with its code.)
# Round 4: the sector-merge seal (LVK_SEAL_SECTORS=1) -- its parity under the
# table tests, then the table bench alternated with the product library, and
# a WRITE_SIZE pass of each.  usage: tools/r04_seal_ab.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/seal_ab}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
bash tools/build_variant.sh sectors -DLVK_SEAL_SECTORS=1 > "$out/build.txt" 2>&1 &&
var=$root/leveldb-rs_amd/lib/variants/liblvgpu_sectors.so &&
LVGPU_EXPERIMENT=1 LVGPU_LIB=$var timeout -k 10 300 python3 -u -m pytest tests/test_table.py -m gpu -x -v \
  --timeout 120 --timeout-method thread > "$out/pytest_table_sectors.txt" 2>&1 &&
echo "variant parity ok" &&
bash tools/ab_table.sh "$out" "sectors:-DLVK_SEAL_SECTORS=1" 3 &&
(cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$root/$out/pmc_prod" -o pmc -- \
   python3 "$root/bench.py" --table --steps 5 --warmup 1 --no-settle --cpu-seconds 0) > "$out/pmc_prod.log" 2>&1 &&
(cd /tmp && LVGPU_EXPERIMENT=1 LVGPU_LIB=$var timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv \
   -d "$root/$out/pmc_var" -o pmc -- python3 "$root/bench.py" --table --steps 5 --warmup 1 --no-settle --cpu-seconds 0) \
   > "$out/pmc_var.log" 2>&1 &&
python3 tools/pmc_summary.py "$out/pmc_prod" "$out/pmc_prod.json" > /dev/null &&
python3 tools/pmc_summary.py "$out/pmc_var" "$out/pmc_var.json" > /dev/null &&
echo "all steps done"
