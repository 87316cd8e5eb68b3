#!/bin/bash
# One GPU pass after a change: the GPU suite, then the default bench line at
# the driver's flags; extra bench.py argument sets follow as NAME:ARGS pairs.
# usage: tools/r03_check.sh OUTDIR [name:"--args" ...]
set -o pipefail
O=${1:-gpurun_out/check}; shift
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest.txt" 2>&1 || { echo PYTEST FAILED; tail -30 "$O/pytest.txt"; exit 1; }
tail -1 "$O/pytest.txt"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$O/default.json" 2> "$O/default.err" || { echo DEFAULT FAILED; tail -20 "$O/default.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open('$O/default.json')); print('default', d['value'], d['roofline']['frac'], d['roofline']['traffic'])"
for spec in "$@"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 300 python bench.py $args > "$O/$name.json" 2> "$O/$name.err" || { echo "$name FAILED"; tail -20 "$O/$name.err"; exit 1; }
  echo "$name: $(head -c 700 "$O/$name.json")"
done
