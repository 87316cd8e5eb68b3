#!/bin/bash
# Round 4: the hinted identity path (uniform, > 1,024 buffers, nothing splits:
# class kernel alone) -- parity tests, then the size sweep and long buffers.
set -o pipefail
O=gpurun_out/r04_ident
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_batch.py tests/test_gpu_stress.py > $O/pytest.log 2>&1 &&
timeout -k 10 240 python -u bench.py --sweep --steps 40 --warmup 20 > $O/sweep.json 2> $O/sweep.err &&
timeout -k 10 240 python -u bench.py --long --steps 40 --warmup 20 > $O/long.json 2> $O/long.err
rc=$?
tail -3 $O/pytest.log
exit $rc
