#!/bin/bash
# Round 5: WAL one-launch scan, global round counters vs own LDS counters
# (variant ns: LVK_WAL_STEAL=0), three interleaved reps; then the host-code
# ASan pass.  usage: tools/r05_run5.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05r6}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
bash tools/build_variant.sh ns -DLVK_WAL_STEAL=0 > "$out/build.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --wal-device --cpu-seconds 0 > "$out/steal_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_ns.so timeout -k 10 200 python3 bench.py --wal-device --cpu-seconds 0 \
    > "$out/ns_$r.json" 2>> "$out/err.txt" || exit 1
done
for f in "$out"/steal_*.json "$out"/ns_*.json; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['roofline']['frac'], d['roofline']['ms_avg'])" "$f"; done
bash tools/r05_asan.sh "$out/asan" && tail -3 "$out/asan/pytest.txt" && tail -2 "$out/asan/stress.txt" &&
echo "all steps done"
