#!/bin/bash
# Round 6 final tree after the seal's explicit-wait change: the GPU suite,
# smoke, three --table runs and the table kernels' stats and FETCH / WRITE.
set -o pipefail
out=${1:-gpurun_out/r06fs}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/pytest_gpu.txt" 2>&1 || { tail -5 "$out/pytest_gpu.txt"; exit 1; }
tail -1 "$out/pytest_gpu.txt"
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.txt" 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --table > "$out/table_$r.json" 2>> "$out/err.txt" || exit 1
done
bash tools/prof_8f.sh "$out/prof8f" table > "$out/prof8f.log" 2>&1 || exit 1
for f in "$out"/table_*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['seal']['frac_of_8TBps'], d['verify']['frac_of_8TBps'])" "$f"; done
