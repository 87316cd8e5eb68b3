#!/bin/bash
# Round 4 second check: the GPU suite, smoke, a 200-trial randomised sweep.
# usage: tools/r04_check2.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r04b}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/pytest.txt" 2>&1 &&
echo "pytest done" &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 &&
LVGPU_STRESS_TRIALS=200 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_stress.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > "$out/stress200.txt" 2>&1 &&
echo "all steps done"
