#!/bin/bash
# Round 5: the WAL one-launch scan with deferred claim reads (tests,
# --wal-device, timeline), then the pipelined host recovery at other chunk
# sizes / copy threads.  usage: tools/r05_run4.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05r5}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out/wal"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wal.py tests/test_wal_log.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > "$out/wal/pytest.txt" 2>&1 &&
timeout -k 10 300 python3 bench.py --wal-device --cpu-seconds 0 > "$out/wal/wal_device.json" 2> "$out/wal/wal_device.err" &&
bash tools/r05_waltrace.sh "$out/wal/trace" &&
tail -c 400 "$out/wal/wal_device.json" &&
python3 -c "import json; d=json.load(open('$out/wal/trace/trace.json')); print({k: d[k] for k in ('end','own_done_last_wave','walk_done_first_wave','walk_done_last_wave','ready','lookback_done')})" &&
bash tools/r05_walhost.sh "$out/walhost" &&
echo "all steps done"
