#!/bin/bash
# Round 6 (2nd): the library bound its worker / copy threads to the GPU's
# socket (bind_thread_to_device, commit a221205, reverted after this A/B:
# with the caller floating it made the host paths slower).  A/B of the
# recovery and host-path lines with LVGPU_THREAD_AFFINITY=0 / 1, floating and
# with the bench process confined to the GPU-local CPUs.
set -o pipefail
out=${1:-gpurun_out/r06aff}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_wal.py tests/test_gpu_batch.py tests/test_teardown.py -x -q -m gpu --timeout 120 --timeout-method thread > "$out/pytest.txt" 2>&1 || { tail -5 "$out/pytest.txt"; exit 1; }
tail -1 "$out/pytest.txt"
local=$(python3 - <<'PY'
import ctypes, glob, os
hip = ctypes.CDLL("libamdhip64.so")
buf = ctypes.create_string_buffer(64)
hip.hipDeviceGetPCIBusId(buf, 64, 0)
print(open(f"/sys/bus/pci/devices/{buf.value.decode().lower()}/local_cpulist").read().strip())
PY
)
echo "local cpus: $local"
for r in 1 2 3; do
  for a in 0 1; do
    LVGPU_THREAD_AFFINITY=$a timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 > "$out/float_aff${a}_$r.json" 2>> "$out/err.txt" || exit 1
  done
  LVGPU_THREAD_AFFINITY=1 timeout -k 10 300 taskset -c "$local" python3 bench.py --wal --cpu-seconds 0 > "$out/local_aff1_$r.json" 2>> "$out/err.txt" || exit 1
done
for a in 0 1; do
  LVGPU_THREAD_AFFINITY=$a timeout -k 10 200 python3 bench.py --e2e > "$out/e2e_aff$a.json" 2>> "$out/err.txt" || exit 1
done
for f in "$out"/float_*.json "$out"/local_*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], 'recovery', d['recovery_pipelined']['GiB_per_s'], 'pinned-log', d['recovery_pipelined_pinned_log']['GiB_per_s'], 'scan', d['scan']['GiB_per_s'], 'reader', d['reader_native']['GiB_per_s'], 'encode', d['encode']['GiB_per_s'])" "$f"; done
for f in "$out"/e2e_*.json; do python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['results'])" "$f"; done
