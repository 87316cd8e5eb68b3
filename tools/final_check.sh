#!/bin/bash
# Final check on the shipped tree: the whole GPU suite, smoke, and
# the driver's default bench line.  usage: tools/final_check.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/final}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/pytest.txt" 2>&1 &&
tail -3 "$out/pytest.txt" &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.txt" 2>&1 &&
timeout -k 10 400 python3 bench.py > "$out/bench.json" 2> "$out/bench.err" &&
python3 -c "import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'])" &&
echo "all steps done"
