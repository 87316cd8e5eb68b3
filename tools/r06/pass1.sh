#!/bin/bash
# Round 6, first GPU pass: tools/r06/first.sh (WAL device tests, --wal-device
# with FETCH/WRITE, the exit probe), bench.py --wal twice (pipelined recovery,
# pageable and pinned log), tools/r06/sst.sh (the SST run-length A/B).
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
mkdir -p gpurun_out/r06wal
bash tools/r06/first.sh gpurun_out/r06first &&
timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 > gpurun_out/r06wal/wal_1.json 2> gpurun_out/r06wal/wal_1.err &&
timeout -k 10 300 python3 bench.py --wal --cpu-seconds 0 > gpurun_out/r06wal/wal_2.json 2> gpurun_out/r06wal/wal_2.err &&
bash tools/r06/sst.sh gpurun_out/r06sst &&
echo pass1 done
