#!/bin/bash
# Round 5: the overlapped WAL scan (path 3: phase A on a CU-masked stream
# beside the framing kernels, then the class kernel with chunked device
# rounds, merged by wal_unsort): WAL GPU tests, then the device bench for
# paths 2 (five-launch) and 3, two interleaved reps, and a kernel trace.
# usage: tools/r05_ovl.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05ovl}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_wal.py -x -q --timeout 300 --timeout-method thread -m gpu \
  > "$out/pytest.txt" 2>&1 || { tail -40 "$out/pytest.txt"; exit 1; }
tail -2 "$out/pytest.txt"
for r in 1 2; do
  for p in 2 3; do
    timeout -k 10 200 python3 bench.py --wal-device --wal-path $p --cpu-seconds 0 > "$out/p${p}_$r.json" 2>> "$out/err.txt" || exit 1
  done
done
for f in "$out"/p*_*.json; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['roofline']['frac'], d['roofline']['ms_avg'], d.get('parity'))" "$f"; done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/$out/prof" -o trace -- python3 "$root/bench.py" --wal-device --wal-path 3 --cpu-seconds 0 --steps 20 --warmup 5 > "$root/$out/prof.json" 2>> "$root/$out/err.txt" || exit 1
cd "$root" && find "$out/prof" -name "*kernel_stats.csv" -exec cp {} "$out/kernel_stats_p3.csv" \; && find "$out/prof" -name "*kernel_trace.csv" -exec python3 tools/ovl_trace.py {} "$out/timeline_p3.txt" \; ; rm -rf "$out/prof"
echo "all steps done"
