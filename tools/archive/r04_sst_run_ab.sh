#!/bin/bash
# (Run once in round 4, profiles/r04/sst_run/; the switch it measured was then retired with its code.)
# Round 4: run-ordered table walk (LVK_SST_RUN = R: a group walks R
# consecutive blocks in consecutive rounds).  Parity of each variant under
# the table tests, the table bench alternated with the product library, and
# a FETCH_SIZE pass of each.  usage: tools/r04_sst_run_ab.sh OUTDIR R1 [R2 ...]
set -o pipefail
out=${1:-gpurun_out/sst_run}; shift
runs=${*:-8 16}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
spec=""
for R in $runs; do
  bash tools/build_variant.sh run$R -DLVK_SST_RUN=$R > "$out/build_run$R.txt" 2>&1 || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$root/leveldb-rs_amd/lib/variants/liblvgpu_run$R.so timeout -k 10 300 \
    python3 -u -m pytest tests/test_table.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$out/pytest_table_run$R.txt" 2>&1 || exit 1
  spec="$spec run$R:-DLVK_SST_RUN=$R"
done
echo "variant parity ok" &&
bash tools/ab_table.sh "$out" "$spec" 3 &&
pmc() { local tag=$1; shift
  (cd /tmp && timeout -s KILL 150 "$@" rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$root/$out/pmc_$tag" -o pmc -- \
     python3 "$root/bench.py" --table --steps 5 --warmup 1 --no-settle --cpu-seconds 0) > "$out/pmc_$tag.log" 2>&1 &&
  python3 tools/pmc_summary.py "$out/pmc_$tag" "$out/pmc_$tag.json" > /dev/null; }
pmc prod env &&
for R in $runs; do
  pmc run$R env LVGPU_EXPERIMENT=1 LVGPU_LIB=$root/leveldb-rs_amd/lib/variants/liblvgpu_run$R.so || exit 1
done &&
echo "all steps done"
