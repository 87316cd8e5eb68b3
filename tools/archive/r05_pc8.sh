#!/bin/bash
# Round 5: the one-launch WAL scan with phase-A first records walked as 8 KiB
# pieces (LVK_PIPE_PIECE=8192) against the product's one-launch and
# five-launch scans, three interleaved reps; the WAL GPU tests on the
# variant; then its phase timeline (timing variant).  usage: tools/r05_pc8.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r05pc8}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
VD=$root/leveldb-rs_amd/lib/variants
bash tools/build_variant.sh pc8 -DLVK_PIPE_PIECE=8192 > "$out/build.txt" 2>&1 || exit 1
bash tools/build_variant.sh pc8t -DLVK_PIPE_PIECE=8192 -DLVK_WAL_PIPE_TRACE=1 >> "$out/build.txt" 2>&1 || exit 1
LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_pc8.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_wal.py tests/test_wal_log.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest_pc8.txt" 2>&1 || { tail -30 "$out/pytest_pc8.txt"; exit 1; }
tail -2 "$out/pytest_pc8.txt"
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --wal-device --wal-path 2 --cpu-seconds 0 > "$out/p2_$r.json" 2>> "$out/err.txt" &&
  timeout -k 10 200 python3 bench.py --wal-device --wal-path 1 --cpu-seconds 0 > "$out/p1_$r.json" 2>> "$out/err.txt" &&
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_pc8.so timeout -k 10 200 python3 bench.py --wal-device --wal-path 1 --cpu-seconds 0 \
    > "$out/pc8_$r.json" 2>> "$out/err.txt" || exit 1
done
for f in "$out"/*_[123].json; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['roofline']['frac'], d['roofline'].get('ms_avg'))" "$f"; done
LVGPU_EXPERIMENT=1 LVGPU_LIB=$VD/liblvgpu_pc8t.so timeout -k 10 300 python3 tools/wal_pipe_trace.py 5 > "$out/trace.json" 2> "$out/trace.err" || exit 1
python3 -c "
import json; d=json.load(open('$out/trace.json'))
for k in ('phaseA_done_last_wave', 'walk_done_first_wave', 'walk_done_last_wave', 'end', 'idle_after_walk'):
    print(k, d[k])"
echo "all steps done"
