#!/bin/bash
# Round 6 final tree, call A: the GPU suite, smoke(), and the --wal-device
# line with its FETCH_SIZE / WRITE_SIZE child passes.
set -o pipefail
out=${1:-gpurun_out/r06fa}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/pytest_gpu.txt" 2>&1 || { tail -5 "$out/pytest_gpu.txt"; exit 1; }
tail -1 "$out/pytest_gpu.txt"
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.txt" 2>&1 || exit 1
timeout -k 10 400 python3 bench.py --wal-device > "$out/wal_device.json" 2> "$out/wal_device.err" || exit 1
python3 -c "import json;d=json.loads(open('$out/wal_device.json').read().splitlines()[-1]);print(json.dumps(d['roofline'],indent=1))"
