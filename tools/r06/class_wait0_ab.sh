#!/bin/bash
# Round 6 (2nd): the explicit folded-batch wait in the class kernel with its
# masked loads (LVK_CLASS_WAIT0=1; with exact loads it measured flat or
# slower, curwait_ab.sh) against the product: C2, C4, C3 via offsets, WAL.
# (The knob lived in commit 061dc0e only.)
set -o pipefail
out=${1:-gpurun_out/r06cw0}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
bash tools/build_variant.sh ccw -DLVK_CLASS_WAIT0=1 > "$out/build.txt" 2>&1 || exit 1
VD=$root/leveldb-rs_amd/lib/variants
LVGPU_STRESS_TRIALS=300 LVGPU_WAL_STRESS_TRIALS=200 LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_ccw.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_batch.py tests/test_gpu_stress.py tests/test_gpu_wal.py tests/test_gpu_wal_stress.py -x -q -m gpu --timeout 120 --timeout-method thread > "$out/pytest_ccw.txt" 2>&1 || { tail -5 "$out/pytest_ccw.txt"; exit 1; }
B="--cpu-seconds 0 --traffic off --c5-strong off"
for r in 1 2; do
  for v in prod ccw; do
    if [ $v = prod ]; then E=""; else E="LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_ccw.so"; fi
    env $E timeout -k 10 300 python3 bench.py --workload c2 --api offsets $B > "$out/c2_${v}_$r.json" 2>> "$out/err.txt" || exit 1
    env $E timeout -k 10 300 python3 bench.py --workload c4 --api offsets $B > "$out/c4_${v}_$r.json" 2>> "$out/err.txt" || exit 1
    env $E timeout -k 10 300 python3 bench.py --workload c3 --api offsets $B > "$out/c3o_${v}_$r.json" 2>> "$out/err.txt" || exit 1
    env $E timeout -k 10 300 python3 bench.py --wal-device --cpu-seconds 0 --traffic off > "$out/wal_${v}_$r.json" 2>> "$out/err.txt" || exit 1
  done
done
python3 - "$out" <<'PY'
import glob, json, os, sys
out = sys.argv[1]
for f in sorted(glob.glob(os.path.join(out, "*.json"))):
    d = json.loads(open(f).read().splitlines()[-1])
    if "seal" in d:
        print(os.path.basename(f), "seal", d["seal"]["frac_of_8TBps"], "verify", d["verify"]["frac_of_8TBps"])
    else:
        print(os.path.basename(f), d["roofline"]["frac"])
PY
