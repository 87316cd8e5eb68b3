#!/bin/bash
# Round 4: the WAL device scan with the CRCs stored by sorted position and
# written in log order by wal_unsort (product) against the class kernel's
# scattered stores (variant nounsort: LVK_WAL_UNSORT=0).  WAL GPU tests, then
# bench --wal-device alternated.  usage: tools/r04_wal_unsort.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/wal_unsort}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_wal.py tests/test_wal_log.py tests/test_wal_boundary.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > "$out/pytest.txt" 2>&1 &&
bash tools/build_variant.sh nounsort -DLVK_WAL_UNSORT=0 > "$out/build.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --wal-device --cpu-seconds 0 > "$out/wal_prod_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_nounsort.so timeout -k 10 200 python3 bench.py --wal-device --cpu-seconds 0 \
    > "$out/wal_nounsort_$r.json" 2>> "$out/err.txt" || exit 1
done &&
echo "all steps done"
