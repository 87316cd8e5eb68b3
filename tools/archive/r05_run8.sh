#!/bin/bash
# Round 5: the full check (GPU suite, smoke, sweep, long, pack probe, gloo8
# rehearsal), the host-code ASan pass, and the pipelined host recovery with 8
# vs 4 staging-copy threads.  usage: tools/r05_run8.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05r9}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
bash tools/r05_check1.sh "$out/check"
echo "check rc=$?"; tail -3 "$out/check/pytest.txt"; cat "$out/check/smoke.txt" 2>/dev/null
bash tools/r05_asan.sh "$out/asan"
echo "asan rc=$?"; tail -2 "$out/asan/pytest.txt"; tail -2 "$out/asan/stress.txt" 2>/dev/null
VD=$root/leveldb-rs_amd/lib/variants
bash tools/build_variant.sh t4 -DLVK_MEMCPY_THREADS=4 > "$out/build_t4.txt" 2>&1 &&
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 > "$out/wal_prod_$r.json" 2>> "$out/wal_err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_t4.so timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 \
    > "$out/wal_t4_$r.json" 2>> "$out/wal_err.txt" || break
done
for f in "$out"/wal_*_*.json; do python3 -c "
import json,sys
for l in open(sys.argv[1]):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[1], d['recovery_pipelined']['GiB_per_s'], d['recovery_pipelined']['parts_ms'], d['reader_native']['ms'])" "$f"; done
echo "all steps done"
