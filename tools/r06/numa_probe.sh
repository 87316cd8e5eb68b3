#!/bin/bash
# Round 6 (2nd): where the pipelined recovery runs on the box -- the CPUs the
# process may use, their NUMA nodes, the GPU's NUMA node -- and the recovery
# line with the process confined to the GPU-local CPUs it may use, against
# the default placement, interleaved.
set -o pipefail
out=${1:-gpurun_out/r06numa}
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
export TMPDIR=/tmp
python3 - > "$out/topo.json" <<'PY'
import glob, json, os
aff = sorted(os.sched_getaffinity(0))
node_of = {}
for d in glob.glob("/sys/devices/system/node/node*"):
    n = int(d.rsplit("node", 1)[1])
    for part in open(d + "/cpulist").read().strip().split(","):
        a, _, b = part.partition("-")
        for c in range(int(a), int(b or a) + 1):
            node_of[c] = n
import ctypes
hip = ctypes.CDLL("libamdhip64.so")
buf = ctypes.create_string_buffer(64)
hip.hipDeviceGetPCIBusId(buf, 64, 0)  # the visible device 0 (the bench's GPU)
bdf = buf.value.decode().lower()
gpus = {bdf: int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read())}
nodes = {}
for c in aff:
    nodes.setdefault(node_of.get(c, -1), []).append(c)
print(json.dumps({"affinity_cpus": len(aff), "nodes_of_affinity": {k: len(v) for k, v in nodes.items()},
                  "gpu_numa": gpus, "n_nodes": len(set(node_of.values())),
                  "local_cpus": ",".join(str(c) for c in aff if node_of.get(c) in set(gpus.values())),
                  "remote_cpus": ",".join(str(c) for c in aff if node_of.get(c) not in set(gpus.values()))}))
PY
python3 -c "import json;d=json.load(open('$out/topo.json'));print(d['gpu_numa'], d['nodes_of_affinity'])"
local=$(python3 -c "import json;print(json.load(open('$out/topo.json'))['local_cpus'])")
remote=$(python3 -c "import json;print(json.load(open('$out/topo.json'))['remote_cpus'])")
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 > "$out/def_$r.json" 2>> "$out/err.txt" || exit 1
  timeout -k 10 300 taskset -c "$local" python3 bench.py --wal --cpu-seconds 0 > "$out/local_$r.json" 2>> "$out/err.txt" || exit 1
  timeout -k 10 300 taskset -c "$remote" python3 bench.py --wal --cpu-seconds 0 > "$out/remote_$r.json" 2>> "$out/err.txt" || exit 1
done
for f in "$out"/def_*.json "$out"/local_*.json "$out"/remote_*.json; do [ -f "$f" ] && python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], d['recovery_pipelined']['GiB_per_s'], d['recovery_pipelined_pinned_log']['GiB_per_s'], d['reader_native']['GiB_per_s'], d['recovery_pipelined']['parts_ms'])" "$f"; done
