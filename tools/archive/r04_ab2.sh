#!/bin/bash
# Round 4, one GPU call: the hash wait-count A/B, then the sorted-walk one.
set -o pipefail
./tools/r04_hash_wait.sh gpurun_out/hash_wait && ./tools/r04_exact_ab.sh gpurun_out/exact_ab 2
