#!/bin/bash
# Round 6 final tree: five bench.py --wal runs in one box (the
# pipelined recovery's min / median over five runs, not a best-of).
set -o pipefail
out=${1:-gpurun_out/r06rec}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
for r in 1 2 3 4 5; do
  timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 > "$out/wal_$r.json" 2>> "$out/err.txt" || exit 1
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['recovery_pipelined']['GiB_per_s'], d['recovery_pipelined_pinned_log']['GiB_per_s'], d['scan_plus_native_reader'])" "$out/wal_$r.json"
done
