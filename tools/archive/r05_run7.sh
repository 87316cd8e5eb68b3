#!/bin/bash
# Round 5: WAL device scan, one-launch vs five-launch path (two interleaved
# reps), the one-launch per-wave timeline, the host-code ASan pass, then the
# full check (GPU suite, smoke, sweep, long, pack probe, gloo8).
# usage: tools/r05_run7.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05r8}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --wal-device --cpu-seconds 0 > "$out/auto_$r.json" 2>> "$out/wal_err.txt" &&
  timeout -k 10 300 python3 bench.py --wal-device --wal-path 2 --cpu-seconds 0 > "$out/p2_$r.json" 2>> "$out/wal_err.txt" || exit 1
done
for f in "$out"/auto_*.json "$out"/p2_*.json; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['roofline']['frac'], d['roofline']['ms_avg'], d['roofline']['kernels'])" "$f"; done
bash tools/r05_waltrace.sh "$out/trace" || exit 1
bash tools/r05_asan.sh "$out/asan"
echo "asan rc=$?"; tail -3 "$out/asan/pytest.txt"; tail -2 "$out/asan/stress.txt" 2>/dev/null
bash tools/r05_check1.sh "$out/check" && tail -3 "$out/check/pytest.txt" && cat "$out/check/smoke.txt" &&
echo "all steps done"
