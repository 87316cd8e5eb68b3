set -o pipefail
o=gpurun_out/exp7; mkdir -p $o
timeout -k 10 400 python3 -m pytest tests -m gpu -x -q > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
for w in c3 c2 c4; do
  timeout -k 10 200 python3 bench.py --workload $w --api offsets --cpu-seconds 0 --traffic off > $o/${w}.json 2>&1 || exit 1
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$o/prof_c3 -o p -- python3 $GRAFT_REPO_ROOT/bench.py --workload c3 --api offsets --steps 50 --warmup 100 --cpu-seconds 0 --traffic off > $GRAFT_REPO_ROOT/$o/prof.log 2>&1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$o/prof_c2 -o p -- python3 $GRAFT_REPO_ROOT/bench.py --workload c2 --api offsets --steps 50 --warmup 100 --cpu-seconds 0 --traffic off > $GRAFT_REPO_ROOT/$o/prof2.log 2>&1 || exit 1
echo done
