#!/bin/bash
# One GPU-box pass of every bench line and kernel profile for the round:
#   bench.py default (C3 strided, headline) at the driver's flags and at the
#   bench defaults, C3 offsets, C2, C4, C5 (8 GiB per GPU) and C5 strong (the
#   64 GiB global batch), the C1 CPU sweep, the host-memory E2E path, the WAL
#   (host and device-resident) / table / hash rows of SURVEY 8f, the 4-64 KiB
#   sweep, few-long-buffer batches, rocprofv3 kernel-trace stats for C3
#   (strided) / C2 / C4 / the WAL device scan / the SST and hash kernels (with
#   FETCH_SIZE / WRITE_SIZE passes) / the few-long-buffer offsets calls, and
#   the N=2 launcher rehearsal (gloo, both ranks on the one GPU).  Every GPU
#   step has its own timeout and the chain stops at the first failure;
#   tools/round_summary.py writes summary.md (events beside rocprof sums).
# usage: tools/measure_round.sh OUTDIR [bench|prof|all]
#   (round 4: the bench lines carry CPU baselines and the default lines a
#   c5_strong sub-record, so the pass is run as two GPU calls: bench, prof)
set -o pipefail
out=${1:-gpurun_out/round}
part=${2:-all}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
b() { local name=$1; shift; timeout -k 10 400 python3 bench.py "$@" > "$out/$name.json" 2> "$out/$name.err"; }
p() { local name=$1; shift
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/$out/prof_$name" -o "$name" -- \
         python3 "$root/bench.py" --steps 50 --warmup 100 --cpu-seconds 0 --traffic off --c5-strong off "$@") > "$out/prof_$name.log" 2>&1 &&
      python3 tools/kstats_steady.py "$(ls "$out/prof_$name"/*kernel_trace.csv | head -n 1)" 50 "$out/prof_${name}_steady.json" > /dev/null; }
bench_part() {
b default_driver --steps 20 --warmup 5 &&
b default &&
b c3_offsets --workload c3 --api offsets --cpu-seconds 5 &&
b c2 --workload c2 --api offsets --cpu-seconds 5 &&
b c4 --workload c4 --api offsets --cpu-seconds 5 &&
b c5 --workload c5 --cpu-seconds 5 &&
b c5_strong --workload c5 --scaling strong --steps 20 --warmup 5 --cpu-seconds 5 &&
timeout -k 10 200 python3 bench.py --e2e > "$out/e2e.json" 2> "$out/e2e.err" &&
timeout -k 10 300 python3 bench.py --c1 > "$out/c1.json" 2> "$out/c1.err" &&
timeout -k 10 300 python3 bench.py --wal > "$out/wal.json" 2> "$out/wal.err" &&
timeout -k 10 300 python3 bench.py --table > "$out/table.json" 2> "$out/table.err" &&
timeout -k 10 300 python3 bench.py --hash > "$out/hash.json" 2> "$out/hash.err" &&
timeout -k 10 300 python3 bench.py --sweep > "$out/sweep.json" 2> "$out/sweep.err" &&
timeout -k 10 300 python3 bench.py --wal-device > "$out/wal_device.json" 2> "$out/wal_device.err" &&
timeout -k 10 300 python3 bench.py --variants > "$out/variants.json" 2> "$out/variants.err" &&
timeout -k 10 300 python3 bench.py --long > "$out/long.json" 2> "$out/long.err"; }
prof_part() {
p c3 &&
p c2 --workload c2 --api offsets &&
p c4 --workload c4 --api offsets &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/$out/prof_wal" -o wal -- \
   python3 "$root/bench.py" --wal-device --steps 50 --warmup 20 --cpu-seconds 0) > "$out/prof_wal.log" 2>&1 &&
python3 tools/kstats_steady.py "$(ls "$out/prof_wal"/*kernel_trace.csv | head -n 1)" 50 "$out/prof_wal_steady.json" > /dev/null &&
bash tools/prof_8f.sh "$out/prof8f" table hash wal &&
bash tools/prof_long.sh "$out/prof_long" &&
LVGPU_BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 --cpu-seconds 2 > "$out/gloo2.json" 2> "$out/gloo2.err" &&
for d in "$out"/prof_*/; do find "$d" -name '*kernel_trace.csv' -size +1M -delete; done; }
case $part in
  bench) bench_part ;;
  prof) prof_part ;;
  *) bench_part && prof_part ;;
esac &&
python3 tools/round_summary.py "$out" > "$out/summary.md" &&
echo "all steps done"
