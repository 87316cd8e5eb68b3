set -o pipefail
O=gpurun_out/r03a; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { echo PYTEST FAILED; tail -30 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
LVGPU_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/gloo2.json 2> $O/gloo2.err || { echo GLOO FAILED; tail -30 $O/gloo2.err; exit 1; }
head -c 600 $O/gloo2.json; echo
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/default.json 2> $O/default.err || { echo DEFAULT FAILED; tail -30 $O/default.err; exit 1; }
head -c 400 $O/default.json; echo
timeout -k 10 120 python bench.py --gpus 2 --steps 5 --warmup 1 --cpu-seconds 0 > $O/nccl2_on_1gpu.json 2> $O/nccl2_on_1gpu.err; echo "nccl2 on 1 gpu rc=$?"; tail -3 $O/nccl2_on_1gpu.err
